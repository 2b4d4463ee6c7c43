#!/bin/bash
# round 6, call j: bwd4 window-group size in the step (the step favours few, long workgroups)
source tools/gpurun_lib.sh
O=$PWD/gpurun_out/r7j
mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 5"
for G in 8 16 32 6 8 16 32 12; do
  DFK_DRPB_G=$G step 300 $B > $O/g${G}_$RANDOM.json 2> $O/g$G.err
done
(cd r5ref && step 300 $B > $O/r5.json 2> $O/r5.err)
