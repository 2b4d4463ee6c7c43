#!/bin/bash
# tile-size A/B of the LDS-DMA GEMM on the mid-size C2 shapes, then the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-wt}
mkdir -p $OUT
for wt in 32 64; do
  DFK_GEMM_WT=$wt timeout -k 10 120 python3 -u tools/gemm_bench.py --only vst2,vst3,vst4,mel1,merge1,w2v,mel3 \
      > $OUT/wt${wt}.txt 2>&1 || { tail -20 $OUT/wt${wt}.txt; exit 1; }
done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
