#!/bin/bash
# weight-gradient split-K depth sweep (tokens per split) on the C2 Linear shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-mink}; mkdir -p $OUT
for mk in 256 512 1024 2048; do
  DFK_DW_MINK=$mk timeout -k 10 200 python3 -u tools/gemm_bench.py > $OUT/mk$mk.txt 2>&1 || { tail -20 $OUT/mk$mk.txt; exit 1; }
done
echo done
