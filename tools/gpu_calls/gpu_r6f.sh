#!/bin/bash
# r6f: shader clock of the PatchEmbed3D forward in-step vs the cold loop (GRBM_GUI_ACTIVE / SQ_BUSY_CYCLES per launch,
# one PMC pass), and the C4 (bf16 / fp8) and C5 bench lines of this build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6f; mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $OUT/clk -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --roofline-iters 6 > $OUT/clk.log 2>&1 || { tail $OUT/clk.log; exit 1; }
python3 - $(find $OUT/clk -name run_counter_collection.csv | head -1) <<'PY'
import csv, sys, collections, statistics
d = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "pe_fwd_kernel" in r["Kernel_Name"]:
        d[int(r.get("Dispatch_Id", 0) or 0)][r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(d)
print("pe_fwd launches", len(ids), "(the last 7 are the cold roofline loop)")
for name, sel in (("in-step", ids[:-7]), ("cold", ids[-7:])):
    g = [d[i]["GRBM_GUI_ACTIVE"] for i in sel]
    b = [d[i]["SQ_BUSY_CYCLES"] for i in sel]
    w = [d[i]["SQ_WAVE_CYCLES"] for i in sel]
    print(f"{name:8s} GRBM_GUI_ACTIVE median {statistics.median(g):.0f}  SQ_BUSY_CYCLES median {statistics.median(b):.0f}  SQ_WAVE_CYCLES median {statistics.median(w):.0f}")
PY
timeout -k 10 400 python3 -u bench.py --config c4 --dtype fp8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c4_fp8.json 2> $OUT/c4_fp8.err || { tail -20 $OUT/c4_fp8.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --config c4 --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c4_bf16.json 2> $OUT/c4_bf16.err || { tail -20 $OUT/c4_bf16.err; exit 1; }
timeout -k 10 500 python3 -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
cut -c1-200 $OUT/c4_fp8.json $OUT/c4_bf16.json $OUT/c5.json
