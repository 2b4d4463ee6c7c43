#!/bin/bash
# r4t: CPB / LN changes — their tests, then the step (3 runs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4t; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_c2.py -k "cpb or layernorm or mel or block" > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -2 $OUT/pt.log
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "run $i: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
