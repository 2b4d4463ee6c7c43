"""MX-fp8 vs bf16 GEMM on the C4 Swin-B video-trunk Linear shapes (B=8): forward (x W^T) and dX (dy W), each with
and without its activation quantisation pass; graph-timed per call.  Prints TFLOP/s per shape and the totals.
Usage: python tools/mx_bench.py [--only vst3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from deepfake_amd import kernels as K  # noqa: E402
from gemm_bench import t  # noqa: E402

B = 8
SHAPES = [  # (name, M tokens, N out, K in): Swin-B, dim 128, 32x224x224 -> 16x56x56 tokens at stage 1
    ("vstB1.qkv", B * 16 * 56 * 56, 384, 128), ("vstB1.fc1", B * 16 * 56 * 56, 512, 128),
    ("vstB1.fc2", B * 16 * 56 * 56, 128, 512),
    ("vstB2.qkv", B * 16 * 28 * 28, 768, 256), ("vstB2.fc1", B * 16 * 28 * 28, 1024, 256),
    ("vstB2.fc2", B * 16 * 28 * 28, 256, 1024),
    ("vstB3.qkv", B * 16 * 14 * 14, 1536, 512), ("vstB3.proj", B * 16 * 14 * 14, 512, 512),
    ("vstB3.fc1", B * 16 * 14 * 14, 2048, 512), ("vstB3.fc2", B * 16 * 14 * 14, 512, 2048),
    ("vstB4.qkv", B * 16 * 7 * 7, 3072, 1024), ("vstB4.fc1", B * 16 * 7 * 7, 4096, 1024),
    ("vstB4.fc2", B * 16 * 7 * 7, 1024, 4096),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    tot = {}
    for name, M, N, Kd in SHAPES:
        if a.only and not any(name.startswith(p) for p in a.only.split(",")):
            continue
        x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, Kd, device="cuda") * Kd ** -0.5)
        wb = w.to(torch.bfloat16)
        dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(M, Kd, device="cuda", dtype=torch.bfloat16)
        xq, wq = K.mx_quant(x), K.mx_quant(w)
        dyq, wtq = K.mx_quant(dy), K.mx_quant(w, transpose=True)
        fl = 2.0 * M * N * Kd
        r = {
            "fwd_bf16": t(lambda: K.linear(x, wb, out=out)),
            "fwd_mx": t(lambda: K.gemm_mx(xq, wq, out=out)),
            "quant_x": t(lambda: K.mx_quant(x)),
            "dx_bf16": t(lambda: K.linear_dx(dy, wb, out=dx)),
            "dx_mx": t(lambda: K.gemm_mx(dyq, wtq, out=dx)),
            "quant_dy": t(lambda: K.mx_quant(dy)),
            "quant_w": t(lambda: K.mx_quant(w)) + t(lambda: K.mx_quant(w, transpose=True)),
        }
        for k, v in r.items():
            tot[k] = tot.get(k, 0.0) + v
        print(f"{name:11s} M={M:6d} N={N:5d} K={Kd:5d}  fwd bf16 {r['fwd_bf16']*1e6:7.1f} us ({fl/r['fwd_bf16']/1e12:6.1f} TF)"
              f"  mx {r['fwd_mx']*1e6:7.1f} us ({fl/r['fwd_mx']/1e12:6.1f} TF) +q {r['quant_x']*1e6:5.1f}"
              f"  | dX bf16 {r['dx_bf16']*1e6:7.1f}  mx {r['dx_mx']*1e6:7.1f} +q {r['quant_dy']*1e6:5.1f}"
              f"  | W quant {r['quant_w']*1e6:5.1f} us", flush=True)
    print("totals (us): " + ", ".join(f"{k} {v*1e6:.1f}" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
