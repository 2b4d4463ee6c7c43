"""Per-(kernel, grid) time per step from a rocprofv3 kernel_trace.csv of bench.py (steps = launches of a
once-per-step marker kernel).   python tools/trace_shapes.py trace.csv [marker] [top]"""
import collections
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "pe_bwd_kernel"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
rows = list(csv.DictReader(open(path)))
steps = sum(1 for r in rows if marker in r["Kernel_Name"])
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    name = r["Kernel_Name"]
    short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
    key = (short, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
    a = agg[key]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"steps (by {marker}): {steps}; total kernel time {tot / steps / 1e3:.2f} ms/step")
for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{us / steps / 1e3:7.3f} ms/step  {n / steps:5.1f}x  avg {us / n:8.1f} us  grid {k[1]}x{k[2]}x{k[3]} wg {k[4]}  {k[0]}")
