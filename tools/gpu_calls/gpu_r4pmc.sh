#!/bin/bash
# r4pmc: counters of the stage-1 fc1 weight gradient (gemm_dma dW) and the stage-1 fc1 + GELU weight-resident
# forward: HBM bytes (FETCH_SIZE x2 on gfx950 / WRITE_SIZE) and SQ issue / wait cycles, one pass per group
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4pmc; mkdir -p $OUT
SQ=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_VMEM,SQ_INSTS_MFMA,SQ_WAVES
for m in dw gelu; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/${m}_t -o run --output-format csv -- python3 tools/dw_one.py $m 401408 384 96 10 > $OUT/${m}_t.log 2>&1 || { tail $OUT/${m}_t.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/${m}_f -o run --output-format csv -- python3 tools/dw_one.py $m 401408 384 96 10 > $OUT/${m}_f.log 2>&1 || { tail $OUT/${m}_f.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/${m}_w -o run --output-format csv -- python3 tools/dw_one.py $m 401408 384 96 10 > $OUT/${m}_w.log 2>&1 || { tail $OUT/${m}_w.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $SQ -d $OUT/${m}_s -o run --output-format csv -- python3 tools/dw_one.py $m 401408 384 96 10 > $OUT/${m}_s.log 2>&1 || { tail $OUT/${m}_s.log; exit 1; }
done
echo done
