#!/bin/bash
# round 6, call g: leaner bwd4 (move-free accumulators, hardware bf16 packing in the slab RMW, pipelined LDS reads)
source tools/gpurun_lib.sh
O=gpurun_out/r7g
mkdir -p $O
step 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wattn.py > $O/wattn.log 2>&1
grep -q "failed" $O/wattn.log && exit 1
step 200 python -u tools/wattn_bench.py 20 > $O/bench_b4.txt 2>&1
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 5"
step 300 $B > $O/b4_1.json 2> $O/b4_1.err
DFK_WATTN_BWD=3 step 300 $B > $O/b3_1.json 2> $O/b3_1.err
step 300 $B > $O/b4_2.json 2> $O/b4_2.err
DFK_WATTN_BWD=3 step 300 $B > $O/b3_2.json 2> $O/b3_2.err
