"""Run one dfk Linear forward shape `iters` times (for rocprofv3 PMC passes):
    python tools/gemm_one.py M N K [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepfake_amd import kernels as K  # noqa: E402

M, N, Kd = (int(v) for v in sys.argv[1:4])
it = int(sys.argv[4]) if len(sys.argv) > 4 else 20
x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, Kd, device="cuda") * Kd ** -0.5).to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(it):
    K.linear(x, w, out=out)
torch.cuda.synchronize()
