#!/bin/bash
# round 6, call i: same-box step A/B: bwd4 (default) / bwd3 / round-5 build; bwd4 window-group sizes
source tools/gpurun_lib.sh
O=$PWD/gpurun_out/r7i
mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 5"
step 300 $B > $O/b4_1.json 2> $O/b4_1.err
DFK_WATTN_BWD=3 step 300 $B > $O/b3_1.json 2> $O/b3_1.err
(cd r5ref && step 300 $B > $O/r5_1.json 2> $O/r5_1.err)
DFK_DRPB_G=2 step 300 $B > $O/g2.json 2> $O/g2.err
DFK_DRPB_G=8 step 300 $B > $O/g8.json 2> $O/g8.err
step 300 $B > $O/b4_2.json 2> $O/b4_2.err
DFK_WATTN_BWD=3 step 300 $B > $O/b3_2.json 2> $O/b3_2.err
(cd r5ref && step 300 $B > $O/r5_2.json 2> $O/r5_2.err)
