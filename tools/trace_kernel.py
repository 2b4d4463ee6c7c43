"""Per-launch-shape durations of one kernel in a rocprofv3 kernel_trace.csv
(grid size distinguishes e.g. the stage-1 window-attention launch from the
other stages), to cross-check bench.py's live HIP-event roofline timing.

    python tools/trace_kernel.py run_kernel_trace.csv 'wattn_fwd_bf16_kernel<32, true, false>'
"""
import csv
import statistics
import sys
from collections import defaultdict

path, name = sys.argv[1], sys.argv[2]
d = defaultdict(list)
for r in csv.DictReader(open(path)):
    if name in r["Kernel_Name"]:
        key = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Workgroup_Size_X"]))
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{name}: launches by (grid_x, grid_y, wg) -> count, mean us, median us")
for k, v in sorted(d.items(), key=lambda kv: -kv[0][0]):
    print(f"  {k}: {len(v):4d}  {statistics.mean(v):9.1f}  {statistics.median(v):9.1f}")
