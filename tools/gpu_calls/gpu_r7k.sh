#!/bin/bash
# round 6, call k: C4 (Swin-B) MX-fp8 per-stage A/B in the full step, plus one kernel trace each of the bf16 and the
# default fp8 step (per-kernel attribution: mx_quant + gemm_mx against the bf16 GEMMs they replace)
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7k
mkdir -p $O
B="python3 -u bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline --roofline-iters 3"
step 400 $B --dtype bf16 > $O/bf16_a.json 2> $O/bf16_a.err
for S in "3" "2" "2,3" "1,2,3" "0,1,2,3"; do
  DFK_FP8_STAGES=$S step 400 $B --dtype fp8 > $O/fp8_s${S//,/}.json 2> $O/fp8_s${S//,/}.err
done
step 400 $B --dtype bf16 > $O/bf16_b.json 2> $O/bf16_b.err
step 400 rocprofv3 --kernel-trace -d $O/tb -o run --output-format csv -- python3 bench.py --config c4 --dtype bf16 \
    --steps 6 --warmup 3 --no-cpu-baseline --roofline-iters 1 > $O/tb.log 2>&1
step 400 rocprofv3 --kernel-trace -d $O/tf -o run --output-format csv -- python3 bench.py --config c4 --dtype fp8 \
    --steps 6 --warmup 3 --no-cpu-baseline --roofline-iters 1 > $O/tf.log 2>&1
python3 tools/step_census.py $(find $O/tb -name run_kernel_trace.csv | head -1) 5 60 > $O/census_bf16.txt
python3 tools/step_census.py $(find $O/tf -name run_kernel_trace.csv | head -1) 5 60 > $O/census_fp8.txt
rm -rf $O/tb $O/tf
head -3 $O/census_bf16.txt $O/census_fp8.txt
