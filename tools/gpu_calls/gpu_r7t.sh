#!/bin/bash
# round 6, call t: a 3-stage LDS ring for the 8-wave 128x64 / 64x128 forward / dX tiles (DFK_DMA_S8W=3; 72 KB of LDS:
# two workgroups per CU instead of three) — isolated shapes, parity, and the step
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7t
mkdir -p $O
G="python3 -u tools/gemm_bench.py"
step 200 $G > $O/base.txt 2>&1
DFK_DMA_S8W=3 step 200 $G > $O/s8w3.txt 2>&1
DFK_DMA_S8W=3 step 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py > $O/ops_s8w3.log 2>&1
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 3"
step 300 $B > $O/base_1.json 2> $O/base_1.err
DFK_DMA_S8W=3 step 300 $B > $O/s8w3_1.json 2> $O/s8w3_1.err
step 300 $B > $O/base_2.json 2> $O/base_2.err
DFK_DMA_S8W=3 step 300 $B > $O/s8w3_2.json 2> $O/s8w3_2.err
tail -n 1 $O/ops_s8w3.log
grep -h total $O/base.txt $O/s8w3.txt
for f in $O/*.json; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$f'.split('/')[-1], d['value'])"; done
