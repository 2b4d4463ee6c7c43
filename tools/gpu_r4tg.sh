#!/bin/bash
# r4tg: weight-gradient split target (DFK_DW_TARGET workgroups) step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4tg; mkdir -p $OUT
for v in 128 96 192 160 128 96 192 160; do
  DFK_DW_TARGET=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "DW_TARGET=$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/ab.txt
done
