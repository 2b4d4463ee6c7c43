"""LayerNorm forward / backward on the C2 step's shapes (graph-timed per call; backward with the slab
partials + column pass).  Usage: python tools/ln_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from deepfake_amd import kernels as K  # noqa: E402
from gemm_bench import t  # noqa: E402

SHAPES = [("vst1", 401408, 96), ("vst2", 100352, 192), ("vst3", 25088, 384), ("vst4", 6272, 768),
          ("mel1", 25088, 128), ("mel3", 1568, 512), ("w2v", 1592, 768), ("mel4", 392, 1024)]


def main():
    tot = [0.0, 0.0, 0.0, 0.0]
    for name, rows, C in SHAPES:
        x = torch.randn(rows, C, device="cuda").to(torch.bfloat16)
        w = torch.ones(C, device="cuda").to(torch.bfloat16)
        b = torch.zeros(C, device="cuda").to(torch.bfloat16)
        dy = torch.randn(rows, C, device="cuda").to(torch.bfloat16)
        y, mean, rstd = K.layernorm_fwd(x, w, b)
        dw = torch.zeros(C, device="cuda")
        db = torch.zeros(C, device="cuda")
        dx = torch.empty_like(x)
        res = torch.randn(rows, C, device="cuda").to(torch.bfloat16)
        f = t(lambda: K.layernorm_fwd(x, w, b))
        fr = t(lambda: K.layernorm_fwd(x, w, b, residual=res))
        bw = t(lambda: K.layernorm_bwd(dy, x, w, mean, rstd, dw, db, dx=dx))
        ba = t(lambda: K.layernorm_bwd(dy, x, w, mean, rstd, dw, db, dx=dx, addend=res))
        tot[0] += f
        tot[1] += bw
        tot[2] += fr
        tot[3] += ba
        mb = rows * C * 2 * 3 / 1e6
        print(f"{name:5s} rows {rows:6d} C {C:4d}  fwd {f*1e6:6.1f} us (+res {fr*1e6:6.1f})  bwd {bw*1e6:6.1f} us "
              f"(+addend {ba*1e6:6.1f}; {mb / (bw * 1e6) * 1e3:6.0f} GB/s of dy + x + dx)", flush=True)
    print(f"totals us: fwd {tot[0]*1e6:.1f} (+res {tot[2]*1e6:.1f}) bwd {tot[1]*1e6:.1f} (+addend {tot[3]*1e6:.1f})",
          flush=True)


if __name__ == "__main__":
    main()
