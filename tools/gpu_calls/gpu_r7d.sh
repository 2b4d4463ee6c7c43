#!/bin/bash
# round 6, call d: bwd4 with hand-counted pass-A memory ops; v6 dead-half skip; parity + timing
source tools/gpurun_lib.sh
O=gpurun_out/r7d
mkdir -p $O
step 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wattn.py > $O/wattn.log 2>&1
grep -q "failed" $O/wattn.log && exit 1
step 200 python -u tools/wattn_bench.py 20 > $O/bench_b4.txt 2>&1
DFK_DRPB_G=1 step 200 python -u tools/wattn_bench.py 20 > $O/bench_b4_g1.txt 2>&1
export TMPDIR=/tmp
WB_SHAPES=vst1 step 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p4 -o run -- python3 -u tools/wattn_bench.py 10 > $O/p4.log 2>&1
step 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vst.py tests/test_gpu_c2.py \
  tests/test_gpu_fused.py tests/test_gpu_ops.py > $O/fused.log 2>&1
step 300 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
