#!/bin/bash
# round 6, call aa: plain small-M input-gradient products (no epilogue, M <= 131072) on hipBLASLt via torch.matmul
# (DFK_DX_BLAS=1) against dfk_gemm — model-level parity with it, and the step
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7aa
mkdir -p $O
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
DFK_DX_BLAS=1 step 500 $T tests/test_gpu_c2.py tests/test_gpu_fused.py tests/test_gpu_vst.py tests/test_gpu_w2v.py tests/test_gpu_trainstep.py > $O/tests.log 2>&1
tail -n 2 $O/tests.log
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 3"
DFK_DX_BLAS=1 step 300 $B > $O/blas_1.json 2> $O/blas_1.err
step 300 $B > $O/base_1.json 2> $O/base_1.err
DFK_DX_BLAS=1 step 300 $B > $O/blas_2.json 2> $O/blas_2.err
step 300 $B > $O/base_2.json 2> $O/base_2.err
for f in $O/*.json; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$f'.split('/')[-1], d['value'])"; done
