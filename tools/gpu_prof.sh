#!/bin/bash
# Profiling pass on the GPU box: kernel-trace stats of the bench step, attention / GEMM micro-benchmarks,
# and separate PMC passes (HBM bytes; SQ issue counters) over the window-attention benchmark.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 120 python3 tools/wattn_bench.py 20 > $OUT/wattn.log 2>&1 || { tail -30 $OUT/wattn.log; exit 1; }
cat $OUT/wattn.log
timeout -k 10 180 python3 tools/gemm_bench.py --torch > $OUT/gemm.log 2>&1 || { tail -30 $OUT/gemm.log; exit 1; }
cat $OUT/gemm.log
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- \
    python3 tools/wattn_bench.py 3 > $OUT/pmc_fetch.log 2>&1 || { tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- \
    python3 tools/wattn_bench.py 3 > $OUT/pmc_write.log 2>&1 || { tail -20 $OUT/pmc_write.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY \
    -d $OUT/pmc_sq -o run --output-format csv -- \
    python3 tools/wattn_bench.py 3 > $OUT/pmc_sq.log 2>&1 || { tail -20 $OUT/pmc_sq.log; exit 1; }
find $OUT -name '*.csv' | head -20
