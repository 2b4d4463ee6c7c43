"""HBM traffic of bench.py's roofline kernel from rocprofv3 PMC counters.

    python tools/roofline_pmc.py run N                 # N launches of bench.roofline_case (profile this)
    python tools/roofline_pmc.py parse FETCH.csv WRITE.csv OUT.json

Each counter runs in its own pass (MI355X_MICROARCH.md, rocprofv3 PMC slots):
    rocprofv3 --pmc FETCH_SIZE -- python3 tools/roofline_pmc.py run 5
    rocprofv3 --pmc WRITE_SIZE -- python3 tools/roofline_pmc.py run 5
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a
wide streaming read, so it is doubled (guide: HBM section).
"""
import csv
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def run(n):
    import torch
    import bench
    from deepfake_amd.models.fused import CONFIGS
    fn, flops, _ = bench.roofline_case(CONFIGS["c2"], 8, torch.bfloat16)
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    print(f"ran {n} launches, {flops:.3e} FLOP each")


def _per_launch(path, counter, kernel):
    vals = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    return statistics.median(vals), len(vals)


def parse(fetch_csv, write_csv, out):
    import bench
    k = bench.ROOFLINE_KERNEL
    fetch_kib, nf = _per_launch(fetch_csv, "FETCH_SIZE", k.rstrip(">"))
    write_kib, nw = _per_launch(write_csv, "WRITE_SIZE", k.rstrip(">"))
    fetch_raw = fetch_kib * 1024
    write = write_kib * 1024
    d = {"kernel": k, "launches": [nf, nw], "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
         "fetch_bytes_raw": fetch_raw, "fetch_bytes_x2": 2 * fetch_raw, "write_bytes": write,
         "bytes_per_launch": 2 * fetch_raw + write,
         "correction": "FETCH_SIZE doubled (MI355X_MICROARCH.md, HBM: on gfx950 FETCH_SIZE reports half the bytes of "
                       "16-B-per-lane streaming reads; the q/k/v token gathers are 16-B loads); WRITE_SIZE as read"}
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]))
    else:
        parse(*sys.argv[2:5])
