#!/bin/bash
# the single-rank capture probe three times in a row (the watchdog race is timing-dependent)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ddpg2; mkdir -p $OUT
export DFK_DDP_FORCE=1 TORCH_NCCL_CUDA_EVENT_CACHE=0
for i in 1 2 3; do
  timeout -k 10 200 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2952$i \
      tools/ddp_graph_probe.py c1 > $OUT/c1_$i.log 2>&1 || { grep -v "frame #" $OUT/c1_$i.log | tail -20; exit 1; }
  grep -v amdgpu $OUT/c1_$i.log | tail -3
done
