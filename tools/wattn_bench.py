"""Time the window-attention kernels at the C2 training shapes (bf16):
forward / backward launch time (HIP events) and MFMA-equivalent TFLOP/s.

    python tools/wattn_bench.py [iters]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepfake_amd import kernels as K  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = 8
# name, dims (B,D,H,W), window, full window, shift, heads, hd, rpb
SHAPES = [
    ("vst1 SW", (B, 16, 56, 56), (8, 7, 7), (8, 7, 7), (4, 3, 3), 3, 32, True),
    ("vst2 SW", (B, 16, 28, 28), (8, 7, 7), (8, 7, 7), (4, 3, 3), 6, 32, True),
    ("vst3 SW", (B, 16, 14, 14), (8, 7, 7), (8, 7, 7), (4, 3, 3), 12, 32, True),
    ("vst4 W", (B, 16, 7, 7), (8, 7, 7), (8, 7, 7), (0, 0, 0), 24, 32, True),
    ("vst4 SWd", (B, 16, 7, 7), (8, 7, 7), (8, 7, 7), (4, 0, 0), 24, 32, True),
    ("mel1 SW", (B, 1, 56, 56), (1, 7, 7), (1, 7, 7), (0, 3, 3), 4, 32, True),
    ("w2v", (B, 1, 1, 199), (1, 1, 199), (1, 1, 199), (0, 0, 0), 12, 64, False),
]


def timed(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(ITERS):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / ITERS * 1e3  # us


def main():
    dt = torch.bfloat16
    only = os.environ.get("WB_SHAPES")   # comma-separated name prefixes (profiling runs)
    shapes = SHAPES + SHAPES[:1]   # vst1 again, clocks warm
    if only:
        shapes = [s for s in SHAPES if any(s[0].startswith(o) for o in only.split(","))]
    for name, dims, win, fw, shift, heads, hd, has_rpb in shapes:
        rows = dims[0] * dims[1] * dims[2] * dims[3]
        C = heads * hd
        qkv = torch.randn(rows, 3 * C, device="cuda").to(dt)
        L = (2 * fw[0] - 1) * (2 * fw[1] - 1) * (2 * fw[2] - 1)
        rpb = torch.randn(L, heads, device="cuda") * 0.3 if has_rpb else None
        N = win[0] * win[1] * win[2]
        nW = 1
        for n, w in zip(dims[1:], win):
            nW *= -(-n // w)
        scale = hd ** -0.5
        out = torch.empty(rows, C, device="cuda", dtype=dt)
        _, lse, tab = K.wattn_fwd(qkv, qkv[:, C:], qkv[:, 2 * C:], 3 * C, dims, win, fw, shift, heads, hd, scale,
                                  rpb=rpb, out=out, return_table=True)
        dout = torch.randn(rows, C, device="cuda").to(dt)
        dqkv = torch.empty_like(qkv)
        drpb = torch.zeros_like(rpb) if rpb is not None else None
        tf = timed(lambda: K.wattn_fwd(qkv, qkv[:, C:], qkv[:, 2 * C:], 3 * C, dims, win, fw, shift, heads, hd, scale,
                                       rpb=rpb, out=out, tab=tab))
        tb = timed(lambda: K.wattn_bwd((qkv, qkv[:, C:], qkv[:, 2 * C:], out, lse, 3 * C, dims, win, fw, shift, heads,
                                        hd, scale, rpb, None), dout, dqkv, dqkv[:, C:], dqkv[:, 2 * C:], 3 * C,
                                       drpb=drpb, tab=tab))
        tb0 = timed(lambda: K.wattn_bwd((qkv, qkv[:, C:], qkv[:, 2 * C:], out, lse, 3 * C, dims, win, fw, shift, heads,
                                         hd, scale, rpb, None), dout, dqkv, dqkv[:, C:], dqkv[:, 2 * C:], 3 * C,
                                        drpb=None, tab=tab)) if rpb is not None else float("nan")
        tt = timed(lambda: K.wattn_fwd(qkv, qkv[:, C:], qkv[:, 2 * C:], 3 * C, dims, win, fw, shift, heads, hd, scale,
                                       rpb=rpb, out=out)) - tf if rpb is not None else float("nan")   # + the table build
        units = dims[0] * nW * heads
        ff = 4.0 * units * N * N * hd
        fb = 10.0 * units * N * N * hd
        print(f"{name:8s} units {units:6d} N {N:4d} fwd {tf:8.1f} us {ff / tf / 1e6:7.1f} TF/s | "
              f"bwd {tb:8.1f} us {fb / tb / 1e6:7.1f} TF/s (no dRPB {tb0:7.1f} us) | table {tt:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
