"""Run one dfk weight-gradient (or weight-resident GELU forward) shape `iters` times, for rocprofv3 PMC passes:
    python tools/dw_one.py dw M N K [iters]      dW[N,K] += dy[M,N]^T x[M,K] (bias gradient fused)
    python tools/dw_one.py gelu M N K [iters]    y = gelu(x w^T + b) with the pre-activation saved"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepfake_amd import kernels as K  # noqa: E402

mode = sys.argv[1]
M, N, Kd = (int(v) for v in sys.argv[2:5])
it = int(sys.argv[5]) if len(sys.argv) > 5 else 10
x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
if mode == "dw":
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    dw = torch.zeros(N, Kd, device="cuda")
    db = torch.zeros(N, device="cuda")
    for _ in range(it):
        K.linear_dw(dy, x, dw, db=db)
else:
    w = (torch.randn(N, Kd, device="cuda") * Kd ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(it):
        K.linear(x, w, b, act=1, aux=aux, out=out)
torch.cuda.synchronize()
