#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5m; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_wattn.py -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
grep "gradient norms\|passed\|failed" $OUT/pytest.log | tail -8
[ $rc -ne 0 ] && { grep -B2 -A20 "^E " $OUT/pytest.log | head -40; exit 1; }
timeout -k 10 200 python -u tools/wattn_bench.py 20 2>&1 | grep fwd | cut -c1-60
