#!/bin/bash
# round 6, call s: SQ / TCC counter passes of the current stage-1 attention kernels (v6 forward, two-pass backward)
source tools/gpurun_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r7s
mkdir -p $O
step 500 bash tools/pmc_wattn.sh fwd wattn_fwd6 1 > $O/fwd.txt 2>&1
step 500 bash tools/pmc_wattn.sh bwd wattn_bwd4 1 > $O/bwd.txt 2>&1
cp -r gpurun_out/pmc_fwd gpurun_out/pmc_bwd $O/ 2>/dev/null
cat $O/fwd.txt $O/bwd.txt
