#!/bin/bash
# r5e: v5 forward ablations (experiment builds), stage-1 launch times
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -f gpurun_out/exp/log.txt
bash tools/exp_run.sh "python -u tools/wattn_bench.py 20" base ABL NOBIAS NOQK NOEXP NOPV NOBIASEXP > /dev/null 2>&1 || { tail -20 gpurun_out/exp/log.txt; exit 1; }
grep "==\|vst1\|vst3" gpurun_out/exp/log.txt
