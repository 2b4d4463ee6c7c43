#!/bin/bash
# small-grid GEMM sweep: LDS stages of the 64x64-tile DMA kernel x automatic split-K on/off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sweep}
mkdir -p $OUT
for st in 2 3 4; do for ns in 0 1; do
  DFK_DMA_S32=$st DFK_GEMM_NOSPLIT=$ns timeout -k 10 120 python3 -u tools/gemm_bench.py --only mel3,w2v,vst3,vst4,mel1 \
      > $OUT/s${st}_ns${ns}.txt 2>&1 || { tail -20 $OUT/s${st}_ns${ns}.txt; exit 1; }
done; done
echo done
