#!/bin/bash
# r4b: tiled-GEMM non-temporal epilogue stores (exp build gemmnt) and LayerNorm-backward block caps, step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4b; mkdir -p $OUT
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$tag: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/ab.txt
}
for i in 1 2; do
  run base DFK_X=0
  run gemmnt DFK_LIB=$PWD/deepfake_amd/libdfk_gemmnt.so
  run ln1024 DFK_LN_BWD_BLOCKS=1024
  run ln4096 DFK_LN_BWD_BLOCKS=4096
done
