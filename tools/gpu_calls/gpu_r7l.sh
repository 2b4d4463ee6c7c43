#!/bin/bash
# round 6, call l: v6 forward with 8 waves per workgroup (W8: one query-block pair per wave, 128 VGPRs -> 4 waves per
# SIMD instead of 3) against the default, its parity tests, and its step A/B; the bench line's new bwd fields
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7l
mkdir -p $O
step 200 python3 -u tools/wattn_bench.py 20 > $O/wb_base.txt 2>&1
DFK_WATTN_W8=1 step 200 python3 -u tools/wattn_bench.py 20 > $O/wb_w8.txt 2>&1
DFK_WATTN_W8=1 step 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wattn.py \
  -k "fwd" > $O/wattn_w8.log 2>&1
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 10"
step 300 $B > $O/base_1.json 2> $O/base_1.err
DFK_WATTN_W8=1 step 300 $B > $O/w8_1.json 2> $O/w8_1.err
step 300 $B > $O/base_2.json 2> $O/base_2.err
DFK_WATTN_W8=1 step 300 $B > $O/w8_2.json 2> $O/w8_2.err
tail -2 $O/wattn_w8.log
head -3 $O/wb_base.txt $O/wb_w8.txt
