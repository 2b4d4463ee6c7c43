#!/bin/bash
# round 6, call n: per-stage window-group rule in the step, G = min(GMAX, units / GMINWG) (C2 units per stage:
# 3072 / 1536 / 768 / 384): 64 -> 8,8,8,6 (default), 32 -> 8,8,8,8, 96 -> 8,8,8,4, 192 -> 8,8,4,2, 384 -> 8,4,2,1
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7n
mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 3"
for W in 64 192 384 32 96 64 192 384; do
  DFK_DRPB_GMINWG=$W step 300 $B > $O/w${W}_$RANDOM.json 2> $O/w$W.err
done
for f in $O/*.json; do python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'): print('$f'.split('/')[-1], json.loads(l)['value'])"; done
