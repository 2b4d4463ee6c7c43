#!/bin/bash
# r5f: attention tests + v4 / v5 (ping-pong) / v5 without ping-pong timings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5f}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wattn.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && { grep -B2 -A30 "^E \|FAILED\|Error" $OUT/pytest.log | head -60; exit 1; }
rm -f gpurun_out/exp/log.txt
DFK_WATTN_V=4 timeout -k 10 200 python -u tools/wattn_bench.py 20 2>&1 | grep "vst\|mel" | sed 's/^/v4 /'
bash tools/exp_run.sh "python -u tools/wattn_bench.py 20" base NOPP > /dev/null 2>&1 || { tail -20 gpurun_out/exp/log.txt; exit 1; }
grep "==\|vst\|mel" gpurun_out/exp/log.txt
