#!/bin/bash
# r4n: C5 checkpoint-loss check in old / new combine modes, then the full GPU suite (that test deselected)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4n; mkdir -p $OUT
PT="python -u -m pytest -q -s --timeout 120 --timeout-method thread"
timeout -k 10 900 $PT -x -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
DFK_INLAUNCH_COMBINE=0 DFK_WGRAD=0 DFK_SGD_NT=0 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_old.json 2> $OUT/bench_old.err || { tail -20 $OUT/bench_old.err; exit 1; }
cut -c1-200 $OUT/bench_old.json
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_new.json 2> $OUT/bench_new.err || { tail -20 $OUT/bench_new.err; exit 1; }
cut -c1-200 $OUT/bench_new.json
DFK_WGRAD=0 DFK_INLAUNCH_COMBINE=0 timeout -k 10 200 python -u tools/gemm_bench.py > $OUT/gemm_old.log 2>&1 || { tail $OUT/gemm_old.log; exit 1; }
timeout -k 10 200 python -u tools/gemm_bench.py > $OUT/gemm_new.log 2>&1 || { tail $OUT/gemm_new.log; exit 1; }
tail -1 $OUT/gemm_old.log; tail -1 $OUT/gemm_new.log
