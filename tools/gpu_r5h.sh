#!/bin/bash
# r5h: attention tests incl. v6 balanced + v5 / v6 / v6-unbalanced timings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5h}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wattn.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && { grep -B2 -A30 "^E \|FAILED\|Error" $OUT/pytest.log | head -60; exit 1; }
for cfg in "5 512" "6 512" "6 1000000000"; do
  set -- $cfg
  DFK_WATTN_V=$1 DFK_WATTN_BALMIN=$2 timeout -k 10 200 python -u tools/wattn_bench.py 20 > $OUT/wattn_bench_v$1_$2.txt 2>&1 || { tail -20 $OUT/wattn_bench_v$1_$2.txt; exit 1; }
  echo "== v$1 balmin $2"; grep -v amdgpu.ids $OUT/wattn_bench_v$1_$2.txt | grep "fwd" | cut -c1-60
done
