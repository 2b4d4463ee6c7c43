#!/bin/bash
# r5b: attention tests (v5 schedules + fallbacks), v4 vs v5 timings, SQ issue counters of both stage-1 launches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5b; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_wattn.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_wattn.log 2>&1; rc=$?
tail -3 $OUT/pytest_wattn.log
[ $rc -ne 0 ] && { grep -B2 -A30 "^E \|FAILED\|Error" $OUT/pytest_wattn.log | head -80; exit 1; }
for v in 4 5; do
  DFK_WATTN_V=$v timeout -k 10 200 python -u tools/wattn_bench.py 20 > $OUT/wattn_bench_v$v.txt 2>&1 || { tail -20 $OUT/wattn_bench_v$v.txt; exit 1; }
  echo "== v$v"; grep -v amdgpu.ids $OUT/wattn_bench_v$v.txt
done
for v in 4 5; do
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  DFK_WATTN_V=$v timeout -s KILL 90 rocprofv3 --pmc $ctr -d $OUT/v${v}p$i -o run --output-format csv -- python3 tools/wattn_pmc.py 1 3 fwd > $OUT/v${v}p$i.log 2>&1 || { tail -5 $OUT/v${v}p$i.log; echo "pass $i failed"; exit 1; }
done
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
for f in sorted(glob.glob(out + '/v*p*/**/run_counter_collection.csv', recursive=True)):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'wattn_fwd' in r['Kernel_Name']:
            d[r['Counter_Name']].append(float(r['Counter_Value']))
    print(f.split('/')[2], {k: '%.4g' % (sum(v) / len(v)) for k, v in d.items()})
PY
