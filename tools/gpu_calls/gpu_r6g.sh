#!/bin/bash
# r6g: weight-gradient split planning knobs in the step (DFK_DW_TARGET workgroups, DFK_DW_MINK tokens per split)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6g; mkdir -p $OUT
run() { timeout -k 10 300 env "$@" python3 -u bench.py --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }; echo "$* $(cut -c90-175 $OUT/b.json)"; }
run DFK_DW_TARGET=256
run DFK_DW_TARGET=512
run DFK_DW_TARGET=384
run DFK_DW_TARGET=256
run DFK_DW_TARGET=512
run DFK_DW_TARGET=384
