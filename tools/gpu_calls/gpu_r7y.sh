#!/bin/bash
# round 6, call y: bwd4's dK / dV order made independent of the unit plan (bitwise the round-robin results): the fp8
# C2 gradient gate that the plan-dependent order tipped (one RPB tensor at 2.007x its MX-emulation error, bound 2x)
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7y
mkdir -p $O
T="python3 -u -m pytest -q --timeout 120 --timeout-method thread"
step 400 $T tests/test_gpu_c4.py tests/test_gpu_wattn.py > $O/tests.log 2>&1
tail -n 3 $O/tests.log
grep -h "fp8 relative L2" $O/tests.log | cut -c1-400
DFK_POSCONV_WN=0 step 300 $T tests/test_gpu_c4.py -k train_grads > $O/c4_torchwn.log 2>&1
tail -n 2 $O/c4_torchwn.log
grep -h "fp8 relative L2" $O/c4_torchwn.log | cut -c1-400
