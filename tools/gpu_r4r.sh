#!/bin/bash
# r4r: LDS-DMA ring depth of the 64x64-tile GEMM (DFK_DMA_S32) on the small-M shapes and in the step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4r; mkdir -p $OUT
for s in 2 3 4; do
  DFK_DMA_S32=$s timeout -k 10 200 python -u tools/gemm_bench.py --only w2v,mel3,vst4 > $OUT/g$s.log 2>&1 || { tail $OUT/g$s.log; exit 1; }
  echo "S32=$s"; grep "M=" $OUT/g$s.log | sed -E 's/ +fwd +[0-9.]+ TF.*\[([0-9]+\/[0-9]+\/[0-9]+) us\].*/ \1/'
done
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for v in "DFK_DMA_S32=2" "DFK_DMA_S32=3" "DFK_DMA_S32=4" "DFK_DMA_S32=2"; do
  env $v timeout -k 10 300 $B > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
