#!/bin/bash
# SQ counters of the LDS-DMA GEMM on two C2 shapes, both tile sizes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-gpmc}; mkdir -p $OUT
C1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_INST_LDS,SQ_WAIT_ANY,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAVES
for wt in 32 64; do for shp in "25088 384 1536" "6272 3072 768" "1592 3072 768"; do
  tag=wt${wt}_$(echo $shp | tr ' ' '_')
  DFK_GEMM_WT=$wt timeout -s KILL 90 rocprofv3 --pmc $C1 -d $OUT/$tag -o run --output-format csv -- python3 tools/gemm_one.py $shp 20 > $OUT/$tag.log 2>&1 || { tail $OUT/$tag.log; exit 1; }
done; done
echo done
