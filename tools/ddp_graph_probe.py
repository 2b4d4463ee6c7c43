"""Single-rank RCCL probe of the captured step's bucket all-reduces (run under torchrun --nproc-per-node 1
with DFK_DDP_FORCE=1): captures TrainStep(graph=True) with the overlapped all-reduces, checks that the
overlapped form was captured, that replayed steps match an eager step with the same reductions
(one rank: sum / 1), and times the graphed C2 step with the reductions in it.
    torchrun --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tools/ddp_graph_probe.py [c1|c2]"""
import os
import sys
import time

import torch
import torch.distributed as dist

os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
os.environ.setdefault("TORCH_FR_BUFFER_SIZE", "256")

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synthetic_batch  # noqa: E402
from deepfake_amd import rng  # noqa: E402
from deepfake_amd.ddp import GradBucketer  # noqa: E402
from deepfake_amd.models.fused import CONFIGS, build_fused  # noqa: E402
from deepfake_amd.optim import FusedSGD  # noqa: E402
from deepfake_amd.params import ParamStore  # noqa: E402
from deepfake_amd.trainer import TrainStep  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c1"
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
cfg = CONFIGS[cfg_name]
B = 8 if cfg_name == "c2" else 2


def make(graph):
    torch.manual_seed(5)
    rng.manual_seed(5, 0)
    model = build_fused(cfg, compute_dtype=torch.bfloat16).cuda()
    model.train()
    store = ParamStore(model, torch.bfloat16)
    bk = GradBucketer(store, bucket_mb=16.0)
    assert bk.enabled, "DFK_DDP_FORCE=1 expected"
    return TrainStep(model, store, FusedSGD(store, 1e-3, 0.9, 1e-4), bk, graph=graph), store


feat, label = synthetic_batch(cfg, B, torch.device("cuda"), 3)
ge, se = make(False)
le = [ge(feat, label)[0].item() for _ in range(3)]   # the eager replica's RCCL works are fresh when the
gg, sg = make(True)                                   # graph replica captures: TrainStep drains the watchdog
lg = [gg(feat, label)[0].item() for _ in range(3)]
for i in range(3):
    print(f"step {i}: eager loss {le[i]:.6f}  graph loss {lg[i]:.6f}", flush=True)
print("captured overlapped all-reduces:", getattr(gg, "captured_overlap", None))
print("captured BN broadcast:", getattr(gg, "captured_bn", None))
d = (se.flat - sg.flat).abs().max().item() / se.flat.abs().max().item()
print(f"max |param diff| / max |param| after 3 steps: {d:.3e}")
assert d < 1e-2, d
if cfg_name == "c2":
    for _ in range(3):
        gg(feat, label)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        gg(feat, label)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    print(f"C2 graphed step with single-rank bucket all-reduces: {dt * 1e3:.2f} ms -> {B / dt:.1f} clips/s")
dist.destroy_process_group()
print("ok")
