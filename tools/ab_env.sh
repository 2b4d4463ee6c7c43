#!/bin/bash
# A/B of one environment knob on the default bench line and the in-step Conv3D launches:
#   bash tools/ab_env.sh TAG VAR VALUE_A VALUE_B
# per value: bench.py (20 steps) and a rocprofv3 kernel trace of bench.py -> pe_instep json.  Each GPU step has
# its own time limit and the chain stops at the first failure.
set -o pipefail
TAG=$1; VAR=$2; A=$3; B=$4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
run() {
  env "$VAR=$1" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$1.json 2> $OUT/bench_$1.err || { tail -20 $OUT/bench_$1.err; return 1; }
  cut -c1-220 $OUT/bench_$1.json
  export "$VAR=$1"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_$1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/trace_$1.log 2>&1 || { tail -20 $OUT/trace_$1.log; return 1; }
  unset "$VAR"
  python3 tools/pe_instep.py $(find $OUT/tr_$1 -name run_kernel_trace.csv | head -1) $OUT/instep_$1.json && cat $OUT/instep_$1.json
}
run "$A" && run "$B"
