"""In-step duration of the fused Conv3D patch embed from a rocprofv3 kernel trace of `bench.py`.

    python tools/pe_instep.py <run_kernel_trace.csv> <out.json> [roofline_iters] [batch] [frames]

bench.py launches pe_fwd_kernel once per training step (warm-up and timed steps, eager or inside the
replayed HIP graph) and then 1 + roofline_iters times back to back for its isolated `roofline_conv3d`
loop, so in trace order the last 1 + roofline_iters launches are the loop and every earlier one ran
inside a step, beside the other branches' kernels.  Algorithmic bytes per launch as in bench.py:
the fp32 clip batch read once + tokens x (96 bf16 + 2 fp32 LN statistics) written.
"""
import csv
import json
import statistics
import sys

PEAK_HBM_GBS = 8000.0


def main():
    src, out = sys.argv[1], sys.argv[2]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    T = int(sys.argv[5]) if len(sys.argv) > 5 else 32
    rows = []
    with open(src) as f:
        for r in csv.DictReader(f):
            if r["Kernel_Name"].startswith("void (anonymous namespace)::pe_fwd_kernel"):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    loop, step = rows[-(iters + 1):], rows[:-(iters + 1)]
    nbytes = B * T * 3 * 224 * 224 * 4 + B * (T // 2) * 56 * 56 * (96 * 2 + 8)

    def summary(rs):
        d = [(e - s) * 1e-3 for s, e in rs]   # us
        med = statistics.median(d)
        return {"launches": len(d), "mean_us": round(statistics.mean(d), 2), "median_us": round(med, 2),
                "min_us": round(min(d), 2), "max_us": round(max(d), 2),
                "achieved_gbs_median": round(nbytes / (med * 1e-6) / 1e9, 1),
                "frac_median": round(nbytes / (med * 1e-6) / 1e9 / PEAK_HBM_GBS, 4)}
    res = {"kernel": "pe_fwd_kernel (fused PatchEmbed3D forward)", "bytes_per_launch": nbytes,
           "peak_gbs": PEAK_HBM_GBS, "source": src,
           "in_step": summary(step) if step else None, "isolated_loop": summary(loop) if loop else None}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
