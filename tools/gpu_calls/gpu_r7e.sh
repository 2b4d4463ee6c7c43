#!/bin/bash
# round 6, call e: tiled dRPB slabs + pipelined bwd4; step-level A/B of this round's switches
source tools/gpurun_lib.sh
O=gpurun_out/r7e
mkdir -p $O
step 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wattn.py > $O/wattn.log 2>&1
grep -q "failed" $O/wattn.log && exit 1
step 200 python -u tools/wattn_bench.py 20 > $O/bench_b4.txt 2>&1
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 5"
step 300 $B > $O/ab_default.json 2> $O/ab_default.err
DFK_COS_DSCORE=0 step 300 $B > $O/ab_nocos.json 2> $O/ab_nocos.err
DFK_WATTN_BWD=3 step 300 $B > $O/ab_bwd3.json 2> $O/ab_bwd3.err
DFK_COS_DSCORE=0 DFK_WATTN_BWD=3 step 300 $B > $O/ab_nocos_bwd3.json 2> $O/ab_nocos_bwd3.err
step 300 $B > $O/ab_default2.json 2> $O/ab_default2.err
