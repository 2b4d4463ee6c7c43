#!/bin/bash
# r4sdw: LDS-DMA ring depth of the 128x128 weight-gradient GEMMs (DFK_DMA_SDW 2 / 3): dW tests, isolated dW, step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4sdw; mkdir -p $OUT
DFK_DMA_SDW=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
for v in 2 3; do
  DFK_DMA_SDW=$v timeout -k 10 200 python -u tools/gemm_bench.py --only vst1,vst2,vst3,mel1,merge1 > $OUT/g_$v.log 2>&1 || { tail $OUT/g_$v.log; exit 1; }
  echo "== SDW=$v"; grep "M=" $OUT/g_$v.log | sed -E 's/ +fwd +[0-9.]+ TF.*\[([0-9]+\/[0-9]+\/[0-9]+) us\].*/ \1/'
done
for v in 2 3 2 3; do
  DFK_DMA_SDW=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "SDW=$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'], d['roofline_dw']['avg_launch_ms'])")" | tee -a $OUT/ab.txt
done
