"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total ms per step."""
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6 / steps:.2f} ms/step over {sum(int(r['Calls']) for r in rows) / steps:.0f} launches/step")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.2f} ms/step {float(r['Percentage']):6.2f}%  calls/step "
          f"{int(r['Calls']) / steps:7.1f} avg {float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:95]}")
