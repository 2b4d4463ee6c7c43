"""Per-step view of a rocprofv3 kernel trace of bench.py: steps are delimited by the SGD kernel (the
last kernel of every training step).  Prints the median step's wall span, the GPU-busy union, time per
queue, and the top kernels by summed duration (averaged over the last --steps steps).

    python tools/trace_steps.py gpurun_out/.../run_kernel_trace.csv [--steps 10] [--top 40]
"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--end-kernel", default="sgd_runs_kernel")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows))
    ends = [e for s, e, n, q in ks if a.end_kernel in n]
    # a step may run several SGD launches (one per contiguous run of parameters): keep the last of each cluster
    marks = [t for i, t in enumerate(ends) if i + 1 == len(ends) or ends[i + 1] - t > 2_000_000]
    marks = marks[-(a.steps + 1):]
    spans, busy, perk, perq = [], [], collections.defaultdict(float), collections.defaultdict(float)
    nsteps = len(marks) - 1
    for i in range(nsteps):
        t0, t1 = marks[i], marks[i + 1]
        seg = [k for k in ks if k[0] >= t0 and k[1] <= t1]
        spans.append((t1 - t0) / 1e6)
        cur_s = cur_e = None
        tot = 0
        for s, e, n, q in seg:
            perk[n] += (e - s) / 1e6 / nsteps
            perq[q] += (e - s) / 1e6 / nsteps
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            tot += cur_e - cur_s
        busy.append(tot / 1e6)
    print(f"{nsteps} steps: span median {statistics.median(spans):.2f} ms, GPU-busy union median "
          f"{statistics.median(busy):.2f} ms, kernel sum {sum(perk.values()):.2f} ms/step")
    print("per queue (ms/step):", {q: round(v, 2) for q, v in sorted(perq.items())})
    for n, v in sorted(perk.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"{v:8.3f} ms  {n[:120]}")


if __name__ == "__main__":
    main()
