#!/bin/bash
# r5x: kernel-trace durations of the dW GEMM with and without its fused bias gradient
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5x; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- python3 tools/dw_db_probe.py 401408 96 96 > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
python3 - $(find $OUT/t -name run_kernel_trace.csv | head -1) <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-30:]:
    print(f"{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3:8.1f} us  {r['Kernel_Name'][:100]}  grid {r.get('Grid_Size_X')}x{r.get('Grid_Size_Y')}x{r.get('Grid_Size_Z')}")
PY
