#!/bin/bash
# r4w: non-temporal output stores (wres write-heavy Linears; tiled GEMM epilogue) -- isolated GEMMs and step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4w; mkdir -p $OUT
for t in base wresnt gemmnt bothnt; do
  if [ $t = base ]; then lib=""; else lib=$PWD/deepfake_amd/libdfk_$t.so; fi
  DFK_LIB=$lib timeout -k 10 200 python -u tools/gemm_bench.py --only vst1,vst2,vst3,mel1,w2v > $OUT/g_$t.log 2>&1 || { tail $OUT/g_$t.log; exit 1; }
  echo "== $t"; grep "M=" $OUT/g_$t.log | sed -E 's/ +fwd +[0-9.]+ TF.*\[([0-9]+\/[0-9]+\/[0-9]+) us\] +gelu\+aux ([0-9]+) us/ \1 gelu \2/'
done
for t in base wresnt gemmnt bothnt base bothnt; do
  if [ $t = base ]; then lib=""; else lib=$PWD/deepfake_amd/libdfk_$t.so; fi
  DFK_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$t: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/ab.txt
done
