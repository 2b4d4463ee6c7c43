#!/bin/bash
# r4v: default small-grid tile rule (8-wave 128x64 / 64x128 for forward / dX) -- full GPU suite + bench A/B vs 64x64
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4v; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
for v in "DFK_GEMM_T32X=0" "DFK_GEMM_T32X=-1" "DFK_GEMM_T32X=0" "DFK_GEMM_T32X=-1"; do
  env $v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/ab.txt
done
