#!/bin/bash
# r4o: per-feature step A/B (SGD NT, in-launch combine, wgrad) + rocprof kernel stats of the all-new build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4o; mkdir -p $OUT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for v in "DFK_SGD_NT=0" "DFK_INLAUNCH_COMBINE=0" "DFK_WGRAD=0" "DFK_SGD_NT=0 DFK_INLAUNCH_COMBINE=0"; do
  env $v timeout -k 10 300 $B > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v: $(cut -c100-175 $OUT/b.json)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $OUT/trace -name 'run_kernel_stats.csv' | head -1) 13 45 > $OUT/kernel_summary.txt
head -40 $OUT/kernel_summary.txt | cut -c1-160
