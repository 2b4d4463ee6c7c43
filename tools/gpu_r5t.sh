#!/bin/bash
# r5t: gradient zeroing after the forward (DFK_ZERO_LATE=1) vs at the step start: bench A/B and the in-step PatchEmbed
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5t; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainstep.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
DFK_ZERO_LATE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_trainstep.py -x -q --timeout 120 --timeout-method thread >> $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
grep passed $OUT/pytest.log
for v in 0 1 0 1; do
DFK_ZERO_LATE=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $OUT/b$v.json 2> $OUT/b$v.err || { tail -20 $OUT/b$v.err; exit 1; }
echo "late=$v $(cut -c90-175 $OUT/b$v.json)"
done
for v in 0 1; do
DFK_ZERO_LATE=$v timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/t$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/t$v.log 2>&1 || { tail -20 $OUT/t$v.log; exit 1; }
python3 tools/pe_instep.py $(find $OUT/t$v -name run_kernel_trace.csv | head -1) $OUT/pe_$v.json > /dev/null && echo "late=$v $(grep -o '"in_step": {[^}]*}' $OUT/pe_$v.json | cut -c1-120)"
done
