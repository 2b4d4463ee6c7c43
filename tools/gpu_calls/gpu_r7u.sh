#!/bin/bash
# round 6, call u: the GEMM epilogue that loads bias / pre-activation / residual before its first store (a load after a
# store waited for every earlier store), against the build before it (expref/libdfk_pre_epi.so via DFK_LIB): the GPU
# tests, isolated GEMM shapes, the bench's roofline_gemm, and the step
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7u
mkdir -p $O
OLD=$PWD/expref/libdfk_pre_epi.so
step 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -n 2 $O/pytest_gpu.log
G="python3 -u tools/gemm_bench.py"
step 200 $G > $O/gb_new.txt 2>&1
DFK_LIB=$OLD step 200 $G > $O/gb_old.txt 2>&1
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 10"
step 300 $B > $O/new_1.json 2> $O/new_1.err
DFK_LIB=$OLD step 300 $B > $O/old_1.json 2> $O/old_1.err
step 300 $B > $O/new_2.json 2> $O/new_2.err
DFK_LIB=$OLD step 300 $B > $O/old_2.json 2> $O/old_2.err
grep -h total $O/gb_new.txt $O/gb_old.txt
for f in $O/*.json; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$f'.split('/')[-1], d['value'], d['roofline_gemm']['avg_launch_ms'], d['roofline_gemm']['frac'])"; done
