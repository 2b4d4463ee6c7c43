#!/bin/bash
# r6a: bias tables only for the occurring shift classes, fewer / longer table workgroups: table build times (HEAD vs new),
# attention tests, bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6a; mkdir -p $OUT
L=$PWD/deepfake_amd
for tag in old new; do
  lib=$L/libdfk_$tag.so; [ $tag = new ] && lib=$L/libdfk.so
  timeout -k 10 200 env DFK_LIB=$lib python -u tools/wattn_bench.py 20 > $OUT/$tag.txt 2>&1 || { tail -20 $OUT/$tag.txt; exit 1; }
  echo "== $tag"; grep -v amdgpu.ids $OUT/$tag.txt
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
echo "$(cut -c90-175 $OUT/b$i.json)"
done
