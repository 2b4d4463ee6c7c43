#!/bin/bash
# r6h: PatchEmbed3D forward with non-temporal input loads (buffer-load aux 2 / 3): the cold roofline_conv3d of bench.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6h; mkdir -p $OUT
L=$PWD/deepfake_amd
for tag in base penta2 penta3 base penta2; do
  lib=$L/libdfk_$tag.so; [ $tag = base ] && lib=$L/libdfk.so
  timeout -k 10 300 env DFK_LIB=$lib python3 -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]); r=d['roofline_conv3d']; print('$tag', d['value'], r['achieved'], r['frac'], r['avg_launch_ms'])"
done
