#!/bin/bash
# One GPU-box pass: parity tests, eager + graph bench (no CPU baseline). Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_eager.log 2>&1 \
    || { tail -40 gpurun_out/bench_eager.log; exit 1; }
tail -2 gpurun_out/bench_eager.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --graph --no-cpu-baseline > gpurun_out/bench_graph.log 2>&1 \
    || { tail -40 gpurun_out/bench_graph.log; exit 1; }
tail -2 gpurun_out/bench_graph.log
