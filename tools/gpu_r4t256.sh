#!/bin/bash
# r4t256: 256x128 8-wave tiles for large grids (DFK_GEMM_T256 = minimum tile count) step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4t256; mkdir -p $OUT
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$tag: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/ab.txt
}
for i in 1 2; do
  run base DFK_X=0
  run t256_512 DFK_GEMM_T256=512
  run t256_1024 DFK_GEMM_T256=1024
done
