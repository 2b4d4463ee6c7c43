#!/bin/bash
# r5a: v4 attention-forward issue counters (VALU vs MFMA issue, waits, LDS) of the stage-1 launch, plus timings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5a; mkdir -p $OUT
timeout -k 10 200 python -u tools/wattn_bench.py 20 > $OUT/wattn_bench.txt 2>&1 || { tail -20 $OUT/wattn_bench.txt; exit 1; }
grep -v amdgpu.ids $OUT/wattn_bench.txt
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MFMA_BF16"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d $OUT/p$i -o run --output-format csv -- python3 tools/wattn_pmc.py 1 3 fwd > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; echo "pass $i failed"; }
done
python3 - "$OUT" wattn_fwd4 <<'PY'
import csv, glob, collections, sys
out, kname = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(out + '/p*/**/run_counter_collection.csv', recursive=True)):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kname in r['Kernel_Name']:
            d[r['Counter_Name']].append(float(r['Counter_Value']))
    print({k: '%.4g' % (sum(v) / len(v)) for k, v in d.items()})
PY
