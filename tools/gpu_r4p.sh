#!/bin/bash
# r4p: step A/B of the SGD store policy and of the opt-in wgrad kernel (combine off); in-step Conv3D for NT on/off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4p; mkdir -p $OUT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for v in "DFK_SGD_NT=1" "DFK_SGD_NT=0" "DFK_WGRAD=1" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=6" "DFK_SGD_NT=1"; do
  env $v timeout -k 10 300 $B > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
for nt in 1 0; do
  export DFK_SGD_NT=$nt
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr$nt -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/trace$nt.log 2>&1 || { tail -20 $OUT/trace$nt.log; exit 1; }
  python3 tools/pe_instep.py $(find $OUT/tr$nt -name run_kernel_trace.csv | head -1) $OUT/instep_nt$nt.json && echo "NT=$nt $(cat $OUT/instep_nt$nt.json | cut -c1-300)"
done
