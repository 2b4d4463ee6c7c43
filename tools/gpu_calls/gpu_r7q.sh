#!/bin/bash
# round 6, call q: the forward / dX GEMMs' automatic split-K in the step (DFK_GEMM_SPLIT_TARGET: workgroups a small
# grid is split up to, default 768; DFK_GEMM_NOSPLIT=1: never), against the default
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7q
mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 3"
step 300 $B > $O/base_1.json 2> $O/base_1.err
DFK_GEMM_SPLIT_TARGET=384 step 300 $B > $O/st384.json 2> $O/st384.err
DFK_GEMM_SPLIT_TARGET=1536 step 300 $B > $O/st1536.json 2> $O/st1536.err
DFK_GEMM_NOSPLIT=1 step 300 $B > $O/nosplit.json 2> $O/nosplit.err
DFK_GEMM_SPLIT_TARGET=512 step 300 $B > $O/st512.json 2> $O/st512.err
step 300 $B > $O/base_2.json 2> $O/base_2.err
for f in $O/*.json; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$f'.split('/')[-1], d['value'])"; done
