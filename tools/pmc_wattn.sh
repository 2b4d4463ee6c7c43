set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 tools/wattn_pmc.py 1 3 fwd > gpurun_out/pmc/p$i.log 2>&1 || { tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv,glob,collections
for f in sorted(glob.glob('gpurun_out/pmc/p*/**/run_counter_collection.csv', recursive=True)):
    d=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'wattn_fwd_tab' in r['Kernel_Name']:
            d[r['Counter_Name']].append(float(r['Counter_Value']))
    print(f, {k: '%.4g' % (sum(v)/len(v)) for k,v in d.items()})
PY
