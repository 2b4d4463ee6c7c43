#!/bin/bash
# round 6, call x: the weight-norm reduce on one workgroup per kernel position (was one thread per position walking all
# 768 partials: 170 us), its parity, and the step against the torch weight-norm ops (DFK_POSCONV_WN=0)
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7x
mkdir -p $O
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
step 400 $T tests/test_gpu_w2v.py tests/test_gpu_c2.py tests/test_gpu_fused.py > $O/tests.log 2>&1
tail -n 2 $O/tests.log
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 3"
step 300 $B > $O/wn_1.json 2> $O/wn_1.err
DFK_POSCONV_WN=0 step 300 $B > $O/torch_1.json 2> $O/torch_1.err
step 300 $B > $O/wn_2.json 2> $O/wn_2.err
DFK_POSCONV_WN=0 step 300 $B > $O/torch_2.json 2> $O/torch_2.err
step 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 6 --warmup 3 --roofline-iters 1 > $O/tr.log 2>&1
python3 tools/step_census.py $(find $O/tr -name run_kernel_trace.csv | head -1) 5 200 > $O/census.txt
rm -rf $O/tr
head -1 $O/census.txt
grep -h "wn_" $O/census.txt | head -4
for f in $O/*.json; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$f'.split('/')[-1], d['value'])"; done
