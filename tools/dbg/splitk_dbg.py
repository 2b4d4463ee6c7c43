"""Debug: dfk_gemm split-K (in-launch combine vs reduce kernel) on a few shapes; prints dw / ref statistics."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepfake_amd import kernels as K  # noqa: E402

for dt in (torch.float32, torch.bfloat16):
    for (M, N, Kd) in [(1000, 288, 96), (1568, 512, 2048), (1592, 768, 3072)]:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(M, Kd, device="cuda", generator=g).to(dt)
        dy = torch.randn(M, N, device="cuda", generator=g).to(dt)
        dw = torch.zeros(N, Kd, device="cuda")
        K.linear_dw(dy, x, dw)
        ref = dy.float().t() @ x.float()
        torch.cuda.synchronize()
        r = (dw / ref)
        print(dt, M, N, Kd, "dw/ref median %.4f min %.4f max %.4f" % (r.median().item(), r.min().item(), r.max().item()),
              "maxerr %.3e" % ((dw - ref).abs().max() / ref.abs().max()).item(), flush=True)
        w = torch.randn(N, Kd, device="cuda", generator=g).to(dt)
        y = K.linear(x, w)
        refy = x.float() @ w.float().t()
        print("   fwd maxerr %.3e" % ((y.float() - refy).abs().max() / refy.abs().max()).item(), flush=True)
