#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5l; mkdir -p $OUT
timeout -k 10 300 python -u tools/wattn_err.py 2>&1 | grep -v amdgpu.ids | tee $OUT/err.txt
