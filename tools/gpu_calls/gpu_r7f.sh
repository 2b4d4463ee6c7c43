#!/bin/bash
# round 6, call f: same-box comparison of this build against the round-5 build (r5ref/, git archive 97635a6)
source tools/gpurun_lib.sh
O=$PWD/gpurun_out/r7f
mkdir -p $O
export TMPDIR=/tmp
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 5"
step 300 $B > $O/cur1.json 2> $O/cur1.err
(cd r5ref && step 300 $B > $O/r5_1.json 2> $O/r5_1.err)
step 300 $B > $O/cur2.json 2> $O/cur2.err
(cd r5ref && step 300 $B > $O/r5_2.json 2> $O/r5_2.err)
P="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --roofline-iters 2"
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pcur -o run -- $P > $O/pcur.log 2>&1
(cd r5ref && step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pr5 -o run -- $P > $O/pr5.log 2>&1)
