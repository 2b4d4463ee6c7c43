#!/bin/bash
# r5v: LayerNorm backward with the two-group form as its own instantiation: ln bench, GPU suite, bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5v; mkdir -p $OUT
timeout -k 10 200 python -u tools/ln_bench.py > $OUT/ln.txt 2>&1 || { tail -20 $OUT/ln.txt; exit 1; }
grep -v amdgpu.ids $OUT/ln.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
echo "$(cut -c90-175 $OUT/b$i.json)"
done
timeout -k 10 200 python -u tools/gemm_bench.py --only w2v,mel3,vst1,vst2 > $OUT/gemm.txt 2>&1 || { tail -20 $OUT/gemm.txt; exit 1; }
grep -v amdgpu.ids $OUT/gemm.txt
