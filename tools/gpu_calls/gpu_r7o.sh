#!/bin/bash
# round 6, call o: weight gradients on 64x64 tiles (DFK_DW_WT=32: 32 KB of LDS per workgroup, up to 4 per CU; isolated
# dW + db 845 -> 777 us over the C2 shapes, call r7m) in the step, against the default 128x128 tiles
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7o
mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 5"
step 300 $B > $O/base_1.json 2> $O/base_1.err
DFK_DW_WT=32 step 300 $B > $O/wt32_1.json 2> $O/wt32_1.err
step 300 $B > $O/base_2.json 2> $O/base_2.err
DFK_DW_WT=32 step 300 $B > $O/wt32_2.json 2> $O/wt32_2.err
DFK_DW_WT=32 DFK_DW_MINK=256 step 300 $B > $O/wt32_k256.json 2> $O/wt32_k256.err
DFK_DW_WT=32 DFK_DW_MINK=1024 step 300 $B > $O/wt32_k1024.json 2> $O/wt32_k1024.err
for f in $O/*.json; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$f'.split('/')[-1], d['value'], d['roofline_dw']['avg_launch_ms'], d['roofline_dw']['frac'])"; done
