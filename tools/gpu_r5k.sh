#!/bin/bash
# r5k: whole-model gradient error (C1 / C2 tensors vs the reference fixtures) under forward v4 / v5 / v6
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5k}; mkdir -p $OUT
for v in 6 4; do
  DFK_WATTN_V=$v timeout -k 10 400 python -u -m pytest "tests/test_gpu_c2.py::test_fused_c2_train_grads" "tests/test_gpu_c2.py::test_fused_c1_grad_tensors" -q -s --timeout 300 --timeout-method thread -k "dt1" > $OUT/c2_v$v.log 2>&1
  echo "== v$v rc=$?"; grep -E "relative L2|error / reference|gradient tensors:|logits rel err|passed|failed" $OUT/c2_v$v.log | cut -c1-220
done
exit 0
