#!/bin/bash
# round 6, call r: HIP stream priorities of the three branch streams in the captured step (DFK_BRANCH_PRIO =
# video,mel,waveform; lower = higher priority), against equal priorities
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7r
mkdir -p $O
step 120 python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" > $O/prio.txt 2>&1
cat $O/prio.txt
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 3"
step 300 $B > $O/base_1.json 2> $O/base_1.err
DFK_BRANCH_PRIO=-1,0,0 step 300 $B > $O/p_v.json 2> $O/p_v.err
DFK_BRANCH_PRIO=0,-1,-1 step 300 $B > $O/p_ma.json 2> $O/p_ma.err
DFK_BRANCH_PRIO=0,-1,0 step 300 $B > $O/p_m.json 2> $O/p_m.err
DFK_BRANCH_PRIO=0,0,-1 step 300 $B > $O/p_a.json 2> $O/p_a.err
step 300 $B > $O/base_2.json 2> $O/base_2.err
for f in $O/*.json; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$f'.split('/')[-1], d['value'])"; done
