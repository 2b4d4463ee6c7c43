#!/bin/bash
# one-launch SGD (dfk_sgd_step_runs): parity tests, then step A/B against the per-run launches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6j; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_regularize.py tests/test_gpu_trainstep.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in 0 1; do
    DFK_SGD_RUNS=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 20 > $OUT/b${v}_$r.json 2> $OUT/b${v}_$r.err || { tail -20 $OUT/b${v}_$r.err; exit 1; }
    echo "runs=$v rep=$r $(cut -c1-190 $OUT/b${v}_$r.json | sed 's/.*"value": \([0-9.]*\).*"ms_per_step": \([0-9.]*\).*/\1 clips\/s \2 ms/')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
grep -i sgd $(find $OUT/trace -name 'run_kernel_stats.csv' | head -1) | cut -c1-200
