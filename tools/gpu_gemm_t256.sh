#!/bin/bash
# GEMM A/B: default tiles vs 256x128 8-wave tiles (2 and 3 LDS stages); op tests first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-t256}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "linear" \
    > $OUT/pytest_ops.log 2>&1 || { tail -30 $OUT/pytest_ops.log; exit 1; }
DFK_GEMM_T256=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "linear" \
    > $OUT/pytest_ops256.log 2>&1 || { tail -30 $OUT/pytest_ops256.log; exit 1; }
tail -1 $OUT/pytest_ops.log $OUT/pytest_ops256.log
timeout -k 10 200 python3 -u tools/gemm_bench.py > $OUT/base.txt 2>&1 || { tail -20 $OUT/base.txt; exit 1; }
DFK_GEMM_T256=0 timeout -k 10 200 python3 -u tools/gemm_bench.py > $OUT/t256_s2.txt 2>&1 || { tail -20 $OUT/t256_s2.txt; exit 1; }
DFK_GEMM_T256=0 DFK_DMA_S128=3 timeout -k 10 200 python3 -u tools/gemm_bench.py > $OUT/t256_s3.txt 2>&1 || { tail -20 $OUT/t256_s3.txt; exit 1; }
echo done
