#!/bin/bash
# r4xcd: XCD-aware column-slice mapping of the weight-resident GEMM -- tests, isolated GEMMs, step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4xcd; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
for t in noxcd base; do
  if [ $t = base ]; then lib=""; else lib=$PWD/deepfake_amd/libdfk_$t.so; fi
  DFK_LIB=$lib timeout -k 10 200 python -u tools/gemm_bench.py --only vst1,vst2,mel1 > $OUT/g_$t.log 2>&1 || { tail $OUT/g_$t.log; exit 1; }
  echo "== $t"; grep "M=" $OUT/g_$t.log | sed -E 's/ +fwd +[0-9.]+ TF.*\[([0-9]+\/[0-9]+\/[0-9]+) us\] +gelu\+aux ([0-9]+) us/ \1 gelu \2/'
done
for t in noxcd base noxcd base; do
  if [ $t = base ]; then lib=""; else lib=$PWD/deepfake_amd/libdfk_$t.so; fi
  DFK_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$t: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/ab.txt
done
