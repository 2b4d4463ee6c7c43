#!/bin/bash
# round 6, call m: weight-gradient GEMM ring depth / tile size A/B (isolated shapes, dW + fused db), the vectorised
# MX transpose quantisation's bit-exact tests, and the dW parity tests under the candidate knobs
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7m
mkdir -p $O
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
step 300 $T tests/test_gpu_mx.py > $O/mx.log 2>&1
tail -2 $O/mx.log
G="python3 -u tools/gemm_bench.py --only vst1,vst2,vst3,mel1,merge1,mel3,w2v"
step 200 $G > $O/base.txt 2>&1
DFK_DMA_SDW=4 step 200 $G > $O/sdw4.txt 2>&1
DFK_DW_WT=32 step 200 $G > $O/wt32_s2.txt 2>&1
DFK_DW_WT=32 DFK_DMA_SDW32=3 step 200 $G > $O/wt32_s3.txt 2>&1
DFK_DW_WT=32 DFK_DMA_SDW32=3 DFK_DW_MINK=1024 step 200 $G > $O/wt32_s3_k1024.txt 2>&1
DFK_DW_WT=32 DFK_DMA_SDW32=4 step 200 $G > $O/wt32_s4.txt 2>&1
step 200 $G > $O/base2.txt 2>&1
DFK_DMA_SDW=4 step 300 $T tests/test_gpu_ops.py -k "dw" > $O/ops_sdw4.log 2>&1
DFK_DW_WT=32 DFK_DMA_SDW32=3 step 300 $T tests/test_gpu_ops.py -k "dw" > $O/ops_wt32.log 2>&1
tail -1 $O/ops_sdw4.log $O/ops_wt32.log
grep -h "total" $O/*.txt
