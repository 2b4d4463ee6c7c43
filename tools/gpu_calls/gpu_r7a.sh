#!/bin/bash
# round 6, call a: logit_scale dscore path, grouped dRPB backward, ADVICE split-K gating test, C1 A/B
source tools/gpurun_lib.sh
O=gpurun_out/r7a
mkdir -p $O
step 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -s tests/test_gpu_ops.py \
  -k "logit_scale or bias_partials" > $O/ops.log 2>&1
step 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wattn.py > $O/wattn.log 2>&1
DFK_DRPB_G=1 step 200 python -u tools/wattn_bench.py 20 > $O/bench_g1.txt 2>&1
step 200 python -u tools/wattn_bench.py 20 > $O/bench_gauto.txt 2>&1
for v in "1 4" "0 4" "1 2" "0 2"; do
  set -- $v
  DFK_COS_DSCORE=$1 DFK_WATTN_V6MIN=$2 step 200 python -u tools/c1_logit_err.py >> $O/c1.log 2>&1
done
step 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_c2.py \
  tests/test_gpu_vst.py > $O/fused.log 2>&1
