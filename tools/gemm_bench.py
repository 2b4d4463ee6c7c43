"""Micro-benchmark of dfk_gemm on the C2 workload's Linear shapes (B=8):
forward (x W^T), dX (dy W) and dW (dy^T x, split-K fp32 atomics); prints
TFLOP/s per shape.  Usage: python tools/gemm_bench.py [--dtype bf16]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepfake_amd import kernels as K  # noqa: E402

SHAPES = [  # (name, M tokens, N out, K in)
    ("vst1.qkv", 401408, 288, 96), ("vst1.fc1", 401408, 384, 96), ("vst1.fc2", 401408, 96, 384),
    ("vst1.proj", 401408, 96, 96), ("vst2.fc1", 100352, 768, 192), ("vst3.fc1", 25088, 1536, 384),
    ("vst3.fc2", 25088, 384, 1536), ("vst4.fc1", 6272, 3072, 768), ("mel1.fc1", 25088, 512, 128),
    ("mel3.fc1", 1568, 2048, 512), ("w2v.qkv", 1592, 2304, 768), ("w2v.fc1", 1592, 3072, 768),
    ("w2v.fc2", 1592, 768, 3072), ("merge1", 100352, 192, 384), ("mel3.proj", 1568, 512, 512),
    ("mel3.fc2", 1568, 512, 2048), ("w2v.proj", 1592, 768, 768),
]


def t(fn, it=10):
    """Per-call GPU time: `it` calls captured in one HIP graph and replayed (no host launch gaps between them)."""
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(it):
                fn()
        g.replay()
        torch.cuda.synchronize()
        s.record()
        g.replay()
        e.record()
    except Exception:   # not capturable: eager calls
        s.record()
        for _ in range(it):
            fn()
        e.record()
    e.synchronize()
    return s.elapsed_time(e) / it / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--torch", action="store_true", help="also time torch (hipBLASLt) for reference")
    ap.add_argument("--only", default="", help="comma-separated shape-name prefixes")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    tot = {"fwd": 0.0, "dx": 0.0, "dw": 0.0}
    for name, M, N, Kd in SHAPES:
        if a.only and not any(name.startswith(p) for p in a.only.split(",")):
            continue
        x = torch.randn(M, Kd, device="cuda").to(dt)
        w = torch.randn(N, Kd, device="cuda").to(dt)
        dy = torch.randn(M, N, device="cuda").to(dt)
        out = torch.empty(M, N, device="cuda", dtype=dt)
        dx = torch.empty(M, Kd, device="cuda", dtype=dt)
        dw = torch.zeros(N, Kd, device="cuda")
        fl = 2.0 * M * N * Kd
        tf = t(lambda: K.linear(x, w, out=out))
        aux = torch.empty(M, N, device="cuda", dtype=dt)
        tg = t(lambda: K.linear(x, w, out=out, act=1, aux=aux))
        tx = t(lambda: K.linear_dx(dy, w, out=dx))
        tw = t(lambda: K.linear_dw(dy, x, dw))
        dbias = torch.zeros(N, device="cuda")
        twb = t(lambda: K.linear_dw(dy, x, dw, dbias))   # with the fused bias gradient (the training step's form)
        tot["fwd"] += tf
        tot["dx"] += tx
        tot["dw"] += tw
        bytes_f = (M * Kd + M * N + N * Kd) * x.element_size()
        print(f"{name:10s} M={M:7d} N={N:5d} K={Kd:5d}  fwd {fl / tf / 1e12:7.1f} TF ({bytes_f / tf / 1e9:6.0f} GB/s)"
              f"  dx {fl / tx / 1e12:7.1f} TF  dw {fl / tw / 1e12:7.1f} TF   [{tf * 1e6:.0f}/{tx * 1e6:.0f}/{tw * 1e6:.0f} us]"
              f"  gelu+aux {tg * 1e6:.0f} us  dw+db {twb * 1e6:.0f} us",
              flush=True)
        if a.torch:
            rf = t(lambda: torch.nn.functional.linear(x, w))
            rx = t(lambda: dy @ w)
            rw = t(lambda: dy.t() @ x)
            print(f"{'  torch':10s} {'':33s}  fwd {fl / rf / 1e12:7.1f} TF {'':13s}  dx {fl / rx / 1e12:7.1f} TF  "
                  f"dw {fl / rw / 1e12:7.1f} TF   [{rf * 1e6:.0f}/{rx * 1e6:.0f}/{rw * 1e6:.0f} us]", flush=True)
    print("total us", {k: round(v * 1e6) for k, v in tot.items()})


if __name__ == "__main__":
    main()
