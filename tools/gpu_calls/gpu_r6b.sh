#!/bin/bash
# r6b: LayerNorm backward of small row counts with few workgroups and atomic dw/db (DFK_LN_SMALL) vs slab + colsum
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6b; mkdir -p $OUT
for n in 0 32 64 128; do
  DFK_LN_SMALL=$n timeout -k 10 200 python -u tools/ln_bench.py > $OUT/ln$n.txt 2>&1 || { tail -20 $OUT/ln$n.txt; exit 1; }
  echo "== small=$n"; grep -v amdgpu.ids $OUT/ln$n.txt | grep -v "^vst[12]"
done
DFK_LN_SMALL=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_regularize.py tests/test_gpu_w2v.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for n in 0 64 0 64; do
DFK_LN_SMALL=$n timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $OUT/b$n.json 2> $OUT/b$n.err || { tail -20 $OUT/b$n.err; exit 1; }
echo "small=$n $(cut -c90-175 $OUT/b$n.json)"
done
