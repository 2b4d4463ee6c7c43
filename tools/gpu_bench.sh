#!/bin/bash
# Round evidence on the GPU box: default bench line (with the CPU baseline), the rocprofv3 kernel-trace
# stats of the same command, and the PMC passes (one counter per pass) for the roofline kernel's traffic.
# usage: bash tools/gpu_bench.sh TAG
set -o pipefail
TAG=${1:-r1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/bench_$TAG
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- \
    python3 tools/roofline_pmc.py run 5 > $OUT/pmc_fetch.log 2>&1 || { tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- \
    python3 tools/roofline_pmc.py run 5 > $OUT/pmc_write.log 2>&1 || { tail -20 $OUT/pmc_write.log; exit 1; }
python3 tools/roofline_pmc.py parse $OUT/pmc_fetch/run_counter_collection.csv \
    $OUT/pmc_write/run_counter_collection.csv $OUT/roofline_pmc.json
