#!/bin/bash
# round 6, call z: the C2 Linear shapes on dfk_gemm against torch (hipBLASLt) for the plain products
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7z
mkdir -p $O
step 300 python3 -u tools/gemm_bench.py --torch > $O/gemm_vs_torch.txt 2>&1
cat $O/gemm_vs_torch.txt
