#!/bin/bash
# quick kernel-time summary of the default bench command: bash tools/gpu_profq.sh TAG
set -o pipefail
TAG=${1:-q}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $OUT/trace -name 'run_kernel_stats.csv' | head -1) 13 45 > $OUT/kernel_summary.txt
cp $(find $OUT/trace -name 'run_kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
head -45 $OUT/kernel_summary.txt | cut -c1-150
