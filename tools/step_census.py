"""Per-step launch census of a training step from a rocprofv3 kernel trace.

rocprofv3's --stats table counts every dispatch of the process (parameter-store setup copies, the eager warm-up
steps, graph capture, the bench's roofline probes) and prof_summary.py divides that by a nominal step count, so
its launches/step overstates the step. This tool cuts the trace at the step's last kernel (the one-launch SGD,
`sgd_runs_kernel`) and reports, for the last N complete steps (the timed graph replays): launches per step,
kernel time per step and per-kernel counts.

    python tools/step_census.py run_kernel_trace.csv [N=5] [top=30] [marker=sgd_runs_kernel]

(marker: any kernel launched once per step, e.g. pe_bwd_kernel for builds before the one-launch SGD)
"""
import collections
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    marker = sys.argv[4] if len(sys.argv) > 4 else "sgd_runs_kernel"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if marker in r[2]]
    if len(ends) < n + 1:
        sys.exit(f"only {len(ends)} {marker} launches in the trace")
    steps = []
    for a, b in zip(ends[-n - 1:-1], ends[-n:]):
        seg = rows[a + 1:b + 1]
        steps.append(seg)
    counts = [len(s) for s in steps]
    ktime = [sum(e - s for s, e, _ in seg) / 1e6 for seg in steps]
    wall = [(seg[-1][1] - seg[0][0]) / 1e6 for seg in steps]
    print(f"steps {n}: launches/step {counts} (median {statistics.median(counts)}), kernel time/step median "
          f"{statistics.median(ktime):.2f} ms, first-to-last kernel median {statistics.median(wall):.2f} ms")
    per = collections.defaultdict(lambda: [0, 0.0])
    for seg in steps:
        for s, e, name in seg:
            k = name.replace("(anonymous namespace)::", "").replace("void ", "")[:90]
            per[k][0] += 1
            per[k][1] += (e - s) / 1e6
    print(f"{'calls/step':>10} {'ms/step':>8}  kernel")
    for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{c / n:10.1f} {t / n:8.3f}  {k}")
    print("by calls:")
    for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{c / n:10.1f} {t / n:8.3f}  {k}")


if __name__ == "__main__":
    main()
