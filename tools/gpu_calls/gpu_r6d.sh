#!/bin/bash
# r6d: automatic split-K of small forward / dX GEMMs on or off (DFK_GEMM_NOSPLIT=1: no slab + reduce launch) and the
# split target, whole-step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6d; mkdir -p $OUT
run() { timeout -k 10 300 env "$@" python3 -u bench.py --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }; echo "$* $(cut -c90-175 $OUT/b.json)"; }
run DFK_GEMM_NOSPLIT=0
run DFK_GEMM_NOSPLIT=1
run DFK_GEMM_SPLIT_TARGET=384
run DFK_GEMM_NOSPLIT=0
run DFK_GEMM_NOSPLIT=1
run DFK_GEMM_SPLIT_TARGET=384
