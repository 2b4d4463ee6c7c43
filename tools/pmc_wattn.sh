# SQ/TCC counter passes (one rocprofv3 run each) over N launches of one window-attention shape.
#   bash tools/pmc_wattn.sh [fwd|bwd] [kernel-name substring] [stage]
set -o pipefail
which=${1:-fwd}; kname=${2:-wattn_fwd_tab}; st=${3:-1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$which; mkdir -p $out
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d $out/p$i -o run --output-format csv -- python3 tools/wattn_pmc.py $st 3 $which > $out/p$i.log 2>&1 || { tail -5 $out/p$i.log; exit 1; }
done
python3 - "$out" "$kname" <<'PY'
import csv, glob, collections, sys
out, kname = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(out + '/p*/**/run_counter_collection.csv', recursive=True)):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kname in r['Kernel_Name']:
            d[r['Counter_Name']].append(float(r['Counter_Value']))
    print({k: '%.4g' % (sum(v) / len(v)) for k, v in d.items()})
PY
