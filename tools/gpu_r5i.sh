#!/bin/bash
# r5i: v6 default (tests) + forward scheduling experiments + backward bias-through-C-input experiment (BWDC)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5i}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wattn.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && { grep -B2 -A30 "^E \|FAILED\|Error" $OUT/pytest.log | head -60; exit 1; }
DFK_LIB=$PWD/deepfake_amd/libdfk_BWDC.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wattn.py -x -q --timeout 120 --timeout-method thread -k bwd > $OUT/pytest_bwdc.log 2>&1; rc=$?
tail -2 $OUT/pytest_bwdc.log
[ $rc -ne 0 ] && { grep -B2 -A30 "^E \|FAILED\|Error" $OUT/pytest_bwdc.log | head -60; exit 1; }
rm -f gpurun_out/exp/log.txt
bash tools/exp_run.sh "python -u tools/wattn_bench.py 20" base SB SGB BWDC > /dev/null 2>&1 || { tail -20 gpurun_out/exp/log.txt; exit 1; }
grep "==\|vst\|mel" gpurun_out/exp/log.txt | cut -c1-120
