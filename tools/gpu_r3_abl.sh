#!/bin/bash
# round-3 first pass: gpu tests, then the attention ablation builds under tools/wattn_bench.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r3a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -5 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
bash tools/exp_run.sh "python -u tools/wattn_bench.py 20" base tabfix nomax noexp tfne tfnenm nods > $OUT/abl.log 2>&1
cat $OUT/abl.log
