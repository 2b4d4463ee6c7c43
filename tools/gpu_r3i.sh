#!/bin/bash
# Round-3 evidence pass: attention A/B against the previous build (libdfk_old.so), all gpu tests, the C2
# bench line + rocprofv3 kernel stats (+ in-step Conv3D from the trace), and a C5 bench line.
#   usage: bash tools/gpu_r3i.sh TAG
set -o pipefail
TAG=${1:-r3i}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -f deepfake_amd/libdfk_old.so ]; then
  bash tools/exp_run.sh "python -u tools/wattn_bench.py 20" old base > $OUT/wattn_ab.txt 2>&1 || { tail -20 $OUT/wattn_ab.txt; exit 1; }
  cat $OUT/wattn_ab.txt
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $OUT/trace -name 'run_kernel_stats.csv' | head -1) 13 45 > $OUT/kernel_summary.txt
head -24 $OUT/kernel_summary.txt
python3 tools/pe_instep.py $(find $OUT/trace -name 'run_kernel_trace.csv' | head -1) $OUT/${TAG}_conv3d_instep.json
timeout -k 10 600 python3 -u bench.py --config c5 --batch 4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -30 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
timeout -k 10 600 python3 -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
