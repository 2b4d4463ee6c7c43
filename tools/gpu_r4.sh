#!/bin/bash
# round-4 GPU pass: a set of steps, each under its own time limit, stopping at the first failure.
#   tools/gpu_r4.sh <outdir> <step>...   steps: mx | c4 | gpu | benchc4 | benchc4bf | bench | smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; mkdir -p $OUT
PT="python -u -m pytest -x -v -s --timeout 120 --timeout-method thread"
for st in "$@"; do
  case $st in
    mx) timeout -k 10 300 $PT tests/test_gpu_mx.py > $OUT/pytest_mx.log 2>&1 || { tail -40 $OUT/pytest_mx.log; exit 1; }
        tail -3 $OUT/pytest_mx.log ;;
    c4) timeout -k 10 400 $PT tests/test_gpu_c4.py > $OUT/pytest_c4.log 2>&1 || { grep -E "rel err|error|PASS|FAIL|Error|assert" $OUT/pytest_c4.log | tail -40; exit 1; }
        grep -E "rel err|L2|: y |PASSED|FAILED" $OUT/pytest_c4.log | tail -30 ;;
    gpu) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
         tail -3 $OUT/pytest_gpu.log ;;
    benchc4) timeout -k 10 400 python -u bench.py --config c4 --dtype fp8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c4_fp8.json 2> $OUT/bench_c4_fp8.err || { tail -20 $OUT/bench_c4_fp8.err; exit 1; }
             cut -c1-400 $OUT/bench_c4_fp8.json ;;
    benchc4bf) timeout -k 10 400 python -u bench.py --config c4 --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c4_bf16.json 2> $OUT/bench_c4_bf16.err || { tail -20 $OUT/bench_c4_bf16.err; exit 1; }
               cut -c1-400 $OUT/bench_c4_bf16.json ;;
    bench) timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
           cut -c1-300 $OUT/bench_c2.json ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
           tail -1 $OUT/smoke.log ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
