#!/bin/bash
# One GPU-box pass of round-5 evidence: (parity tests,) the default bench line with the CPU baseline, the
# rocprofv3 kernel-trace stats of the same bench command (+ the in-step Conv3D launches), the FETCH / WRITE PMC
# passes of the roofline kernel, and FETCH / WRITE PMC passes of the bench command for the in-step Conv3D.
# Each GPU step has its own time limit; the chain stops at the first failure.
#   usage: bash tools/gpu_round5.sh TAG [skip-tests] [skip-cpu] [pe-pmc] [c4] [c5]
set -o pipefail
TAG=${1:-r5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $OUT/trace -name 'run_kernel_stats.csv' | head -1) 13 45 > $OUT/kernel_summary.txt
python3 tools/pe_instep.py $(find $OUT/trace -name "run_kernel_trace.csv" | head -1) $OUT/${TAG}_conv3d_instep.json
head -30 $OUT/kernel_summary.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_f -o run --output-format csv -- python3 tools/roofline_pmc.py run 5 > $OUT/pmc_f.log 2>&1 || { tail $OUT/pmc_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_w -o run --output-format csv -- python3 tools/roofline_pmc.py run 5 > $OUT/pmc_w.log 2>&1 || { tail $OUT/pmc_w.log; exit 1; }
python3 tools/roofline_pmc.py parse $(find $OUT/pmc_f -name run_counter_collection.csv) $(find $OUT/pmc_w -name run_counter_collection.csv) $OUT/${TAG}_wattn_fwd_pmc.json
# the bench line below cites this run's PMC and in-step files: place them where bench.py reads them (box copy)
mkdir -p profiles/r5 && cp $OUT/${TAG}_wattn_fwd_pmc.json profiles/r5/r5_wattn_fwd_pmc.json
cp $OUT/${TAG}_conv3d_instep.json profiles/r5/r5_conv3d_instep.json
CPU=""
[ "$3" == "skip-cpu" ] && CPU="--no-cpu-baseline"
timeout -k 10 500 python3 -u bench.py $CPU > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
if [ "$4" == "pe-pmc" ]; then
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pe_f -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --roofline-iters 6 > $OUT/pe_f.log 2>&1 || { tail $OUT/pe_f.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum -d $OUT/pe_w -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --roofline-iters 6 > $OUT/pe_w.log 2>&1 || { tail $OUT/pe_w.log; exit 1; }
  python3 tools/pe_pmc.py $(find $OUT/pe_f -name run_counter_collection.csv) $(find $OUT/pe_w -name run_counter_collection.csv) > $OUT/${TAG}_conv3d_pmc.txt
  cat $OUT/${TAG}_conv3d_pmc.txt
fi
if [ "$5" == "c4" ]; then
  timeout -k 10 400 python3 -u bench.py --config c4 --dtype fp8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${TAG}_c4_fp8_bench_line.json 2> $OUT/c4_fp8.err || { tail -20 $OUT/c4_fp8.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --config c4 --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${TAG}_c4_bf16_bench_line.json 2> $OUT/c4_bf16.err || { tail -20 $OUT/c4_bf16.err; exit 1; }
  cut -c1-160 $OUT/${TAG}_c4_fp8_bench_line.json $OUT/${TAG}_c4_bf16_bench_line.json
fi
if [ "$6" == "c5" ]; then
  timeout -k 10 500 python3 -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/${TAG}_c5_bench_line.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
  cut -c1-160 $OUT/${TAG}_c5_bench_line.json
fi
timeout -k 10 300 python3 -u tools/determinism_probe.py c2 bf16 2 > $OUT/determinism_c2_bf16.txt 2>&1 || { tail -20 $OUT/determinism_c2_bf16.txt; exit 1; }
head -30 $OUT/determinism_c2_bf16.txt
