#!/bin/bash
# GEMM A/B on the GPU box: op tests through the LDS-DMA kernel, then the C2 Linear shapes with the DMA
# kernel (3 and 2 LDS stages) and with the register-staged kernel.   usage: bash tools/gpu_gemm_ab.sh TAG
set -o pipefail
TAG=${1:-gemm}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "linear" \
    > $OUT/pytest_ops.log 2>&1 || { tail -30 $OUT/pytest_ops.log; exit 1; }
tail -2 $OUT/pytest_ops.log
timeout -k 10 200 python3 -u tools/gemm_bench.py > $OUT/dma3.txt 2>&1 || { tail -20 $OUT/dma3.txt; exit 1; }
DFK_DMA_S64=2 DFK_DMA_S32=2 timeout -k 10 200 python3 -u tools/gemm_bench.py > $OUT/dma2.txt 2>&1 || { tail -20 $OUT/dma2.txt; exit 1; }
DFK_GEMM_DMA=0 timeout -k 10 200 python3 -u tools/gemm_bench.py --torch > $OUT/reg.txt 2>&1 || { tail -20 $OUT/reg.txt; exit 1; }
echo done
