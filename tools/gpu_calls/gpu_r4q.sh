#!/bin/bash
# r4q: how many parallel streams the HIP graph executor gives the replayed step, and step time vs that count
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4q; mkdir -p $OUT
AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x7fffffff timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --roofline-iters 1 > $OUT/log_b.json 2> $OUT/amdlog.txt
echo "log rc=$?"; grep -a -m8 -i -E "max streams|parallel streams|max_streams|hipGraph\]" $OUT/amdlog.txt | cut -c1-200
rm -f $OUT/amdlog.txt
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for v in "DFK_NONE=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "DEBUG_HIP_FORCE_GRAPH_QUEUES=8"; do
  env $v timeout -k 10 300 $B > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
