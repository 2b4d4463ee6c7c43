#!/bin/bash
# r5t: where the step graph zeroes the gradients (DFK_ZERO_MODE 0 start / 1 after the forward / 2 side stream):
# train-step parity, bench A/B, in-step PatchEmbed3D; LayerNorm bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5t; mkdir -p $OUT
timeout -k 10 200 python -u tools/ln_bench.py > $OUT/ln_new.txt 2>&1 || { tail -20 $OUT/ln_new.txt; exit 1; }
grep -v amdgpu.ids $OUT/ln_new.txt
for m in 1 2; do
DFK_ZERO_MODE=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_trainstep.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest$m.log 2>&1 || { tail -30 $OUT/pytest$m.log; exit 1; }
grep passed $OUT/pytest$m.log
done
for v in 0 1 2 0 1 2; do
DFK_ZERO_MODE=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $OUT/b$v.json 2> $OUT/b$v.err || { tail -20 $OUT/b$v.err; exit 1; }
echo "zero_mode=$v $(cut -c90-175 $OUT/b$v.json)"
done
for v in 0 1 2; do
DFK_ZERO_MODE=$v timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/t$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/t$v.log 2>&1 || { tail -20 $OUT/t$v.log; exit 1; }
python3 tools/pe_instep.py $(find $OUT/t$v -name run_kernel_trace.csv | head -1) $OUT/pe_$v.json > /dev/null
python3 -c "import json; d=json.load(open('$OUT/pe_$v.json')); print('zero_mode=$v in-step pe_fwd', d['in_step'])"
done
