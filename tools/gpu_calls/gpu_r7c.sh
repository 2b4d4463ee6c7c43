#!/bin/bash
# round 6, call c: the two-pass attention backward (bwd4): parity, then timing against bwd3, G=1 / auto
source tools/gpurun_lib.sh
O=gpurun_out/r7c
mkdir -p $O
step 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wattn.py -k "bwd" > $O/wattn.log 2>&1
grep -q " passed" $O/wattn.log || exit 1
grep -q "failed" $O/wattn.log && exit 1
step 200 python -u tools/wattn_bench.py 20 > $O/bench_b4.txt 2>&1
DFK_DRPB_G=1 step 200 python -u tools/wattn_bench.py 20 > $O/bench_b4_g1.txt 2>&1
DFK_WATTN_BWD=3 step 200 python -u tools/wattn_bench.py 20 > $O/bench_b3.txt 2>&1
export TMPDIR=/tmp
WB_SHAPES=vst1 step 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p4 -o run -- python3 -u tools/wattn_bench.py 10 > $O/p4.log 2>&1
step 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vst.py tests/test_gpu_c2.py \
  tests/test_gpu_fused.py > $O/fused.log 2>&1
