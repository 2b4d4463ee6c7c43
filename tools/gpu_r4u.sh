#!/bin/bash
# r4u: 8-wave 128x64 / 64x128 tiles for the small-grid GEMMs (DFK_GEMM_T32X), isolated and in the step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4u; mkdir -p $OUT
timeout -k 10 200 env DFK_GEMM_T32X=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k fwd_bwd > $OUT/pt.log 2>&1 || { tail -20 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
for t in 0 1 2; do
  DFK_GEMM_T32X=$t timeout -k 10 200 python -u tools/gemm_bench.py --only w2v,mel3,vst4,vst3,mel1 > $OUT/g$t.log 2>&1 || { tail $OUT/g$t.log; exit 1; }
  echo "T32X=$t"; grep "M=" $OUT/g$t.log | sed -E 's/ +fwd +[0-9.]+ TF.*\[([0-9]+\/[0-9]+\/[0-9]+) us\].*/ \1/'; tail -1 $OUT/g$t.log
done
for v in "DFK_GEMM_T32X=0" "DFK_GEMM_T32X=1" "DFK_GEMM_T32X=2"; do
  env $v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
