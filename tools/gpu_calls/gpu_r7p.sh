#!/bin/bash
# round 6, call p: the weight-gradient split planner's workgroup target in the step (DFK_DW_TARGET, default 256: the
# split count of a skinny dW is about target / output tiles), and the window-group rule 8,8,8,4 (GMINWG 96) again
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7p
mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 5"
step 300 $B > $O/base_1.json 2> $O/base_1.err
DFK_DW_TARGET=128 step 300 $B > $O/t128.json 2> $O/t128.err
DFK_DW_TARGET=512 step 300 $B > $O/t512.json 2> $O/t512.err
DFK_DW_TARGET=192 step 300 $B > $O/t192.json 2> $O/t192.err
DFK_DRPB_GMINWG=96 step 300 $B > $O/w96.json 2> $O/w96.err
step 300 $B > $O/base_2.json 2> $O/base_2.err
for f in $O/*.json; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$f'.split('/')[-1], d['value'], d['roofline_dw']['avg_launch_ms'], d['roofline_dw']['frac'])"; done
