"""dW GEMM with and without the fused bias gradient (linear_dw(..., db)) on one shape, eager, for a rocprofv3
kernel trace: python tools/dw_db_probe.py M N K"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from deepfake_amd import kernels as K  # noqa: E402

M, N, Kd = (int(v) for v in sys.argv[1:4])
x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
dw = torch.zeros(N, Kd, device="cuda")
db = torch.zeros(N, device="cuda")
for i in range(6):
    K.linear_dw(dy, x, dw)
    K.linear_dw(dy, x, dw, db)
torch.cuda.synchronize()
print("ok")
