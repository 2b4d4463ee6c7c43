#!/bin/bash
# r5z: drpb_from_ds loads in flight (8 / 16) and non-temporal loads: attention backward with / without dRPB
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5z; mkdir -p $OUT
L=$PWD/deepfake_amd
for tag in base dsnt base dsnt; do
  lib=$L/libdfk_$tag.so; [ $tag = base ] && lib=$L/libdfk.so
  timeout -k 10 200 env DFK_LIB=$lib python -u tools/wattn_bench.py 20 > $OUT/$tag.txt 2>&1 || { tail -20 $OUT/$tag.txt; exit 1; }
  echo "== $tag"; grep -v amdgpu.ids $OUT/$tag.txt | head -4
done
