#!/bin/bash
# round 6, call b: where the dRPB time goes (kernel trace, G=1 vs auto), the ONES forward A/B, aten census
source tools/gpurun_lib.sh
O=gpurun_out/r7b
mkdir -p $O
export TMPDIR=/tmp
WB_SHAPES=vst1 DFK_DRPB_G=1 step 200 rocprofv3 --kernel-trace --stats -d $O/g1 -o run -- python3 -u tools/wattn_bench.py 10 > $O/g1.log 2>&1
WB_SHAPES=vst1 step 200 rocprofv3 --kernel-trace --stats -d $O/g4 -o run -- python3 -u tools/wattn_bench.py 10 > $O/g4.log 2>&1
DFK_WATTN_ONES=1 step 200 python -u tools/wattn_bench.py 20 > $O/bench_ones.txt 2>&1
step 200 python -u tools/wattn_bench.py 20 > $O/bench_base.txt 2>&1
DFK_WATTN_ONES=1 step 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wattn.py \
  -k "fwd" > $O/wattn_ones.log 2>&1
step 300 python -u tools/aten_census.py c2 > $O/census.txt 2>&1
