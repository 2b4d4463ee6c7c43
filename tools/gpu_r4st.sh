#!/bin/bash
# r4st: automatic split-K target of small-grid GEMMs (DFK_GEMM_SPLIT_TARGET) step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4st; mkdir -p $OUT
for v in 768 384 1536 768 384 1536; do
  DFK_GEMM_SPLIT_TARGET=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "SPLIT_TARGET=$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/ab.txt
done
