#!/bin/bash
# r5g: attention tests incl. v6 (16x16x32) + v5 / v6 timings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5g}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wattn.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && { grep -B2 -A30 "^E \|FAILED\|Error" $OUT/pytest.log | head -60; exit 1; }
for v in 5 6; do
  DFK_WATTN_V=$v timeout -k 10 200 python -u tools/wattn_bench.py 20 > $OUT/wattn_bench_v$v.txt 2>&1 || { tail -20 $OUT/wattn_bench_v$v.txt; exit 1; }
  echo "== v$v"; grep -v amdgpu.ids $OUT/wattn_bench_v$v.txt | grep "fwd"
done
