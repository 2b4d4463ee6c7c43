#!/bin/bash
# r4tg4: weight-gradient split target at C4 (Swin-B, bf16) step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4tg4; mkdir -p $OUT
for v in 256 160 256 160; do
  DFK_DW_TARGET=$v timeout -k 10 300 python3 -u bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "C4 DW_TARGET=$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/ab.txt
done
