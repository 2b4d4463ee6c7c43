#!/bin/bash
# round 6, call v: bwd4 unit assignment planned per window (DP over unit counts per wave, costs DFK_B4_COST) against
# round robin (DFK_B4_SCHED=0): attention parity, the isolated backward, the step
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7v
mkdir -p $O
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
step 400 $T tests/test_gpu_wattn.py tests/test_gpu_vst.py tests/test_gpu_c2.py > $O/tests.log 2>&1
tail -n 2 $O/tests.log
W="python3 -u tools/wattn_bench.py 20"
DFK_B4_SCHED=0 WB_SHAPES=vst1,vst2,vst3,vst4 step 200 $W > $O/wb_rr.txt 2>&1
WB_SHAPES=vst1,vst2,vst3,vst4 step 200 $W > $O/wb_dp43.txt 2>&1
DFK_B4_COST=3,2 WB_SHAPES=vst1,vst2,vst3,vst4 step 200 $W > $O/wb_dp32.txt 2>&1
DFK_B4_COST=1,1 WB_SHAPES=vst1,vst2,vst3,vst4 step 200 $W > $O/wb_dp11.txt 2>&1
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 10"
step 300 $B > $O/dp_1.json 2> $O/dp_1.err
DFK_B4_SCHED=0 step 300 $B > $O/rr_1.json 2> $O/rr_1.err
step 300 $B > $O/dp_2.json 2> $O/dp_2.err
DFK_B4_SCHED=0 step 300 $B > $O/rr_2.json 2> $O/rr_2.err
grep -h vst $O/wb_*.txt
for f in $O/*.json; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); r=d['roofline_attn_bwd']; print('$f'.split('/')[-1], d['value'], r['avg_launch_ms'], r['frac'], r.get('group4'))"; done
