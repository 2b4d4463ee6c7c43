"""Micro-benchmark of the LayerNorm kernels at the C2 step's row counts (bf16): time and HBM GB/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepfake_amd import kernels as K  # noqa: E402

SHAPES = [(401408, 96), (100352, 192), (100352, 384), (25088, 384), (25088, 768), (6272, 768), (25088, 128),
          (6272, 512), (1568, 512), (1568, 2048), (1592, 768)]


def timed(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it * 1e3


for rows, C in SHAPES:
    x = torch.randn(rows, C, device="cuda").to(torch.bfloat16)
    w = torch.ones(C, device="cuda", dtype=torch.bfloat16)
    b = torch.zeros(C, device="cuda", dtype=torch.bfloat16)
    y, mean, rstd = K.layernorm_fwd(x, w, b)
    dy = torch.randn_like(x)
    dw = torch.zeros(C, device="cuda")
    db = torch.zeros(C, device="cuda")
    dx = torch.empty_like(x)
    tf = timed(lambda: K.layernorm_fwd(x, w, b, out=y))
    tb = timed(lambda: K.layernorm_bwd(dy, x, w, mean, rstd, dw, db, dx=dx))
    nb = rows * C * 2
    print(f"rows {rows:7d} C {C:5d}  fwd {tf:7.1f} us {2 * nb / tf / 1e3:6.0f} GB/s | bwd {tb:7.1f} us "
          f"{3 * nb / tb / 1e3:6.0f} GB/s", flush=True)
