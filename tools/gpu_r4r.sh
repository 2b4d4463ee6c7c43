#!/bin/bash
# r4r: LDS-DMA ring depth of the 64x64-tile GEMM (DFK_DMA_S32) on the small-M shapes and in the step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4r; mkdir -p $OUT
for s in 2 3 4; do
  DFK_DMA_S32=$s timeout -k 10 200 python -u tools/gemm_bench.py --only w2v,mel3,vst4 > $OUT/g$s.log 2>&1 || { tail $OUT/g$s.log; exit 1; }
  echo "S32=$s"; grep "M=" $OUT/g$s.log | sed -E 's/ +fwd +[0-9.]+ TF.*\[([0-9]+\/[0-9]+\/[0-9]+) us\].*/ \1/'
done
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for v in "DFK_DMA_S32=2" "DFK_DMA_S32=3" "DFK_DMA_S32=4" "DFK_DMA_S32=2"; do
  env $v timeout -k 10 300 $B > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --copy-inputs > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
echo "copy-inputs: $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python3 tools/pe_instep.py $(find $OUT/tr -name run_kernel_trace.csv | head -1) $OUT/instep.json && python3 -c "import json;d=json.load(open('$OUT/instep.json'));print('pe in-step', d['in_step']['median_us'], 'isolated', d['isolated_loop']['median_us'])"
timeout -k 10 400 python3 -u bench.py --config c5 --batch 8 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c5_b8.json 2> $OUT/c5_b8.err || { tail -5 $OUT/c5_b8.err; exit 1; }
echo "c5 b8: $(python3 -c "import json;d=json.load(open('$OUT/c5_b8.json'));print(d['value'], d['ms_per_step'])")"
