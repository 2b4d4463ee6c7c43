#!/bin/bash
# One GPU-box pass of round evidence: parity tests, the default bench line (with CPU baseline), and the
# rocprofv3 kernel-trace stats of the same bench command.  Each GPU step has its own time limit; the
# chain stops at the first failure.   usage: bash tools/gpu_round.sh TAG [skip-tests] [skip-cpu]
set -o pipefail
TAG=${1:-r2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
CPU=""
[ "$3" == "skip-cpu" ] && CPU="--no-cpu-baseline"
timeout -k 10 500 python3 -u bench.py $CPU > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $OUT/trace -name 'run_kernel_stats.csv' | head -1) 13 45 > $OUT/kernel_summary.txt
head -40 $OUT/kernel_summary.txt
