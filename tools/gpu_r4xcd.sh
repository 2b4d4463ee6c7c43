#!/bin/bash
# r4xcd: XCD-aware column-slice mapping of the weight-resident GEMM (lib noxcd: off) and XCD-grouped splits of
# the atomic weight-gradient GEMMs (DFK_DW_XCD=0: off) -- tests, isolated GEMMs, step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4xcd; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_fused.py tests/test_gpu_c2.py > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$tag: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'], d['roofline_dw']['avg_launch_ms'])")" | tee -a $OUT/ab.txt
}
for i in 1 2; do
  run base DFK_X=0
  run bothoff DFK_DW_XCD=0 DFK_LIB=$PWD/deepfake_amd/libdfk_noxcd.so
done
