#!/bin/bash
# r4s: LayerNorm backward block cap sweep (isolated), then the step at the best caps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4s; mkdir -p $OUT
for c in 2048 512 256 128; do
  DFK_LN_BWD_BLOCKS=$c timeout -k 10 120 python -u tools/ln_bench.py > $OUT/ln$c.log 2>&1 || { tail $OUT/ln$c.log; exit 1; }
  echo "cap $c"; cat $OUT/ln$c.log | grep -v amdgpu.ids
done
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for v in "DFK_LN_BWD_BLOCKS=2048" "DFK_LN_BWD_BLOCKS=512" "DFK_LN_BWD_BLOCKS=256"; do
  env $v timeout -k 10 300 $B > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
