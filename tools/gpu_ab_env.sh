#!/bin/bash
# bench A/B of one tuning environment variable: bash tools/gpu_ab_env.sh TAG VAR=VALUE
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 20 > $OUT/base.json 2>/dev/null && \
env $2 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 20 > $OUT/var.json 2>/dev/null && \
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 20 > $OUT/base2.json 2>/dev/null && \
python3 -c "
import json
for f in ('base','var','base2'):
    d=json.load(open(f'$OUT/{f}.json')); print(f, d['value'], d['ms_per_step'])"
