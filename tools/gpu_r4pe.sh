#!/bin/bash
# r4pe: software-pipelined PatchEmbed3D backward -- patch-embed / C2 / fused tests, in-step time, step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4pe; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vst.py tests/test_gpu_c2.py tests/test_gpu_fused.py > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
for t in peold base peold base; do
  if [ $t = base ]; then lib=""; else lib=$PWD/deepfake_amd/libdfk_$t.so; fi
  DFK_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$t: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --roofline-iters 2 > $OUT/tr.log 2>&1 || { tail -20 $OUT/tr.log; exit 1; }
python3 - $(find $OUT/tr -name run_kernel_trace.csv | head -1) <<'PY'
import csv, sys
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000 for r in csv.DictReader(open(sys.argv[1])) if 'pe_bwd' in r['Kernel_Name']]
print('pe_bwd launches', len(d), 'us', [round(x, 1) for x in d])
PY
