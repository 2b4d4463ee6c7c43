#!/bin/bash
# r4w12: 192-channel wave tiles for the K = 96 weight-resident GEMMs without residual / dGELU (DFK_WRES_W12=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4w12; mkdir -p $OUT
DFK_WRES_W12=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
for v in 0 1; do
  DFK_WRES_W12=$v timeout -k 10 200 python -u tools/gemm_bench.py --only vst1 > $OUT/g_$v.log 2>&1 || { tail $OUT/g_$v.log; exit 1; }
  echo "== W12=$v"; grep "M=" $OUT/g_$v.log | sed -E 's/ +fwd +[0-9.]+ TF.*\[([0-9]+\/[0-9]+\/[0-9]+) us\] +gelu\+aux ([0-9]+) us/ \1 gelu \2/'
done
for v in 0 1 0 1; do
  DFK_WRES_W12=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "W12=$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/ab.txt
done
