#!/bin/bash
# r5j: C1 bf16 train-step gradient norms under each forward version (which change moved logit_scale's error)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5j}; mkdir -p $OUT
for v in 6 5 4; do
  DFK_WATTN_V=$v timeout -k 10 300 python -u -m pytest "tests/test_gpu_fused.py::test_fused_c1_train_step" -x -q -s --timeout 120 --timeout-method thread > $OUT/c1_v$v.log 2>&1
  echo "== v$v rc=$?"; grep "gradient norms" $OUT/c1_v$v.log
done
exit 0
