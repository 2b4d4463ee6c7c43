"""Time the bench's CPU baseline (oracle C2 train step, B=2) at several torch thread counts on the GPU box."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

for n in [int(a) for a in sys.argv[1:]] or [16, len(os.sched_getaffinity(0))]:
    t0 = time.time()
    r = bench.cpu_baseline("c2", 1, n)
    print(f"threads {n}: {r['sample']} ({time.time() - t0:.1f} s wall)", flush=True)
