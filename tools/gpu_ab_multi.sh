#!/bin/bash
# bench A/B of several tuning environments against the default, base first and last:
#   bash tools/gpu_ab_multi.sh TAG "VAR=V [VAR=V]" ["VAR=V" ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for v in "" "$@" ""; do
  i=$((i+1))
  env $v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 20 > $OUT/v$i.json 2>$OUT/v$i.err || { tail $OUT/v$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/v$i.json')); print('[$v]', d['value'], d['ms_per_step'])" | tee -a $OUT/ab.txt
done
