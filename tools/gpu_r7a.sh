#!/bin/bash
# round 6, call a: logit_scale dscore path + ADVICE split-K gating test + C1 A/B
set -o pipefail
mkdir -p gpurun_out/r7a
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -s tests/test_gpu_ops.py \
  -k "logit_scale or bias_partials" > gpurun_out/r7a/ops.log 2>&1 || exit 1
for v in "1 4" "0 4" "1 2" "0 2"; do
  set -- $v
  DFK_COS_DSCORE=$1 DFK_WATTN_V6MIN=$2 $T 200 python -u tools/c1_logit_err.py >> gpurun_out/r7a/c1.log 2>&1 || exit 1
done
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_c2.py \
  tests/test_gpu_vst.py > gpurun_out/r7a/fused.log 2>&1 || exit 1
