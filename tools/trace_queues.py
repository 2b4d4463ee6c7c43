"""Per-HW-queue kernel time inside one graph-replayed step of a rocprofv3 kernel trace (the three branch
streams land on different queues): python tools/trace_queues.py trace.csv [marker]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "sgd_kernel"
# one step period: between consecutive patch-embed backward launches (once per step)
starts = [int(r["Start_Timestamp"]) for r in rows if "pe_bwd_kernel" in r["Kernel_Name"]]
if len(starts) < 3:
    sys.exit("not enough steps")
a, b = starts[-3], starts[-2]
busy = collections.defaultdict(float)
top = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if a <= s < b:
        q = r["Queue_Id"]
        busy[q] += (e - s) / 1e3
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        top[q][n] += (e - s) / 1e3
print(f"step span {(b - a) / 1e3:.1f} us")
for q, t in sorted(busy.items()):
    print(f"queue {q}: {t:9.1f} us of kernels")
    for n, v in sorted(top[q].items(), key=lambda kv: -kv[1])[:8]:
        print(f"      {v:8.1f}  {n}")

# union of busy intervals (any queue) vs the per-queue sums: how much the branch streams overlap
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if a <= int(r["Start_Timestamp"]) < b)
union, cur_s, cur_e = 0, None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
print(f"busy union {union / 1e3:.1f} us; sum over queues {sum(busy.values()):.1f} us; idle {(b - a - union) / 1e3:.1f} us")
