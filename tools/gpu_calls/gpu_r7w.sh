#!/bin/bash
# round 6, call w: the positional conv's weight norm fused into two kernel pairs (PosConvWNFn) — the GPU tests, and
# the step against the torch weight-norm ops (DFK_POSCONV_WN=0)
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7w
mkdir -p $O
step 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -n 2 $O/pytest_gpu.log
grep -h "weight_norm" $O/pytest_gpu.log | head -3
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 3"
step 300 $B > $O/wn_1.json 2> $O/wn_1.err
DFK_POSCONV_WN=0 step 300 $B > $O/torch_1.json 2> $O/torch_1.err
step 300 $B > $O/wn_2.json 2> $O/wn_2.err
DFK_POSCONV_WN=0 step 300 $B > $O/torch_2.json 2> $O/torch_2.err
step 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 6 --warmup 3 --roofline-iters 1 > $O/tr.log 2>&1
python3 tools/step_census.py $(find $O/tr -name run_kernel_trace.csv | head -1) 5 60 > $O/census.txt
rm -rf $O/tr
head -1 $O/census.txt
for f in $O/*.json; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$f'.split('/')[-1], d['value'])"; done
