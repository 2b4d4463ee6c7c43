#!/bin/bash
# round 6, call h: bwd3 without the slab RMW and with batched K gathers; full GPU suite; same-box r5 comparison
source tools/gpurun_lib.sh
O=$PWD/gpurun_out/r7h
mkdir -p $O
export TMPDIR=/tmp
step 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
grep -q " failed\|error" $O/pytest_gpu.log && { tail -30 $O/pytest_gpu.log; exit 1; }
step 200 python -u tools/wattn_bench.py 20 > $O/wattn_bench.txt 2>&1
B="python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --roofline-iters 5"
step 300 $B > $O/cur1.json 2> $O/cur1.err
(cd r5ref && step 300 $B > $O/r5_1.json 2> $O/r5_1.err)
step 300 $B > $O/cur2.json 2> $O/cur2.err
(cd r5ref && step 300 $B > $O/r5_2.json 2> $O/r5_2.err)
P="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --roofline-iters 2"
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pcur -o run -- $P > $O/pcur.log 2>&1
