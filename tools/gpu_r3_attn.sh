#!/bin/bash
# Round-3 attention pass: gpu tests, bench + kernel stats, then SQ counter passes of the stage-1 forward and
# backward.  Each GPU step has its own limit; the chain stops at the first failure.
#   usage: bash tools/gpu_r3_attn.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $OUT/trace -name 'run_kernel_stats.csv' | head -1) 13 45 > $OUT/kernel_summary.txt
head -24 $OUT/kernel_summary.txt
timeout -k 10 300 python -u tools/wattn_bench.py 20 > $OUT/wattn_bench.txt 2>&1 || { tail $OUT/wattn_bench.txt; exit 1; }
grep -v amdgpu.ids $OUT/wattn_bench.txt
bash tools/pmc_wattn.sh fwd wattn_fwd3 1 > $OUT/pmc_fwd.txt 2>&1 || { tail $OUT/pmc_fwd.txt; exit 1; }
cat $OUT/pmc_fwd.txt
bash tools/pmc_wattn.sh bwd wattn_bwd3 1 > $OUT/pmc_bwd.txt 2>&1 || { tail $OUT/pmc_bwd.txt; exit 1; }
cat $OUT/pmc_bwd.txt
