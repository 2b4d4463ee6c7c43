"""Bisect HIP-graph capture of the training step: capture progressively larger
pieces (forward only, forward+backward, full step) on a given config."""
import faulthandler
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.enable()

from deepfake_amd.models.fused import CONFIGS, build_fused  # noqa: E402
from deepfake_amd.params import ParamStore  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c1"
what = sys.argv[2] if len(sys.argv) > 2 else "fwd"
cfg = CONFIGS[cfg_name]
dt = torch.bfloat16
m = build_fused(cfg, compute_dtype=dt).cuda()
m.train()
store = ParamStore(m, dt)
B = 2
x = (torch.randn(B, cfg["T"], 3, cfg["H"], cfg["W"], device="cuda"), torch.randn(B, 3, 224, 224, device="cuda"),
     torch.randn(B, 16000 * cfg["seconds"], device="cuda"))
y = torch.ones(B, device="cuda")
lossF = torch.nn.BCELoss()


def body():
    p = m(x)
    if what == "fwd":
        return p
    loss = lossF(p.float(), y)
    loss.backward()
    return loss


print("eager", flush=True)
r = body()
torch.cuda.synchronize()
del r
print("eager ok; capturing", what, flush=True)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        out = body()
torch.cuda.current_stream().wait_stream(s)
print("captured", flush=True)
g.replay()
torch.cuda.synchronize()
print("replay ok", float(out.float().sum()), flush=True)
