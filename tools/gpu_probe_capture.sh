cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/probe
DFK_DEBUG_WATCHDOG=1 DFK_DDP_FORCE=1 TORCH_NCCL_CUDA_EVENT_CACHE=0 TORCH_FR_BUFFER_SIZE=256 timeout -k 10 150 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 tools/ddp_graph_probe.py c1 > gpurun_out/probe/probe.log 2>&1; echo rc=$?
grep -v "^frame\|^E1017" gpurun_out/probe/probe.log | head -60
