#!/bin/bash
# r5y: weight gradients through fp32 split slabs + a phase-parallel reduce (DFK_DW_SLAB=1) vs split atomics
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5y; mkdir -p $OUT
timeout -k 10 200 python -u tools/gemm_bench.py --only vst1,vst2,vst3,mel1,mel3 > $OUT/atomic.txt 2>&1 || { tail -20 $OUT/atomic.txt; exit 1; }
DFK_DW_SLAB=1 timeout -k 10 200 python -u tools/gemm_bench.py --only vst1,vst2,vst3,mel1,mel3 > $OUT/slab.txt 2>&1 || { tail -20 $OUT/slab.txt; exit 1; }
echo "== atomic"; grep -v amdgpu.ids $OUT/atomic.txt | cut -c1-40,100-200; echo "== slab"; grep -v amdgpu.ids $OUT/slab.txt | cut -c1-40,100-200
DFK_DW_SLAB=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "dw or linear or gemm" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in 0 1; do
DFK_DW_SLAB=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $OUT/b$v.json 2> $OUT/b$v.err || { tail -20 $OUT/b$v.err; exit 1; }
echo "slab=$v $(cut -c90-175 $OUT/b$v.json)"
done
