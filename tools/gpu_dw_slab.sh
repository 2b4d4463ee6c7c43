#!/bin/bash
# A/B of weight-gradient split-K: fp32 atomics (default) vs fp32 slab partials + reduce, and split depths.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/dwslab; mkdir -p $OUT
for cfg in "0 256" "4 256" "8 256" "16 256" "0 512" "0 1024"; do
  set -- $cfg
  echo "== DFK_DW_SLAB=$1 DFK_DW_MINK=$2" | tee -a $OUT/dw.txt
  DFK_DW_SLAB=$1 DFK_DW_MINK=$2 timeout -k 10 120 python3 -u tools/gemm_bench.py >> $OUT/dw.txt 2>&1 || exit 1
done
grep -E "==|total" $OUT/dw.txt
