#!/bin/bash
# quick GPU pass: all gpu tests (stop at first failure), then the attention micro-benchmark
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-quick}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} \
    > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && { grep -B2 -A30 "^E \|FAILED\|Error" $OUT/pytest_gpu.log | head -60; exit 1; }
timeout -k 10 300 python -u tools/wattn_bench.py 20 2>&1 | grep -v amdgpu.ids | tee $OUT/wattn_bench.txt
