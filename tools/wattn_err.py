"""Attention forward error against an fp32 reference for each kernel version (bf16 inputs, same data).

    python tools/wattn_err.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from deepfake_amd import kernels as K  # noqa: E402
from test_gpu_wattn import ref_attention  # noqa: E402

CASES = [  # name, dims, window, shift, heads, rpb scale, qk scale, bias offset
    ("vst3", (2, 16, 14, 14), (8, 7, 7), (4, 3, 3), 12, 0.02, 1.0, 0.0),
    ("vst1", (1, 16, 56, 56), (8, 7, 7), (4, 3, 3), 3, 0.02, 1.0, 0.0),
    ("mel-like", (2, 1, 56, 56), (1, 7, 7), (0, 3, 3), 4, 3.0, 6.0, 8.0),
]


def main():
    hd = 32
    for name, dims, win, shift, heads, rs, qks, boff in CASES:
        g = torch.Generator(device="cuda").manual_seed(1)
        rows = dims[0] * dims[1] * dims[2] * dims[3]
        C = heads * hd
        qkv = torch.randn(rows, 3 * C, device="cuda", generator=g)
        qkv[:, :C] *= qks
        qkv = qkv.to(torch.bfloat16)
        L = (2 * win[0] - 1) * (2 * win[1] - 1) * (2 * win[2] - 1)
        rpb = torch.randn(L, heads, device="cuda", generator=g) * rs + boff
        ref = ref_attention(qkv, [torch.zeros(C, device="cuda")] * 3, dims, win, win, shift, heads, hd, hd ** -0.5, rpb)
        line = f"{name:9s}"
        for v in (4, 5, 6):
            K.wattn_fwd_policy(v, -2)
            out, _ = K.wattn_fwd(qkv, qkv[:, C:], qkv[:, 2 * C:], 3 * C, dims, win, win, shift, heads, hd, hd ** -0.5,
                                 rpb=rpb)
            d = (out.float() - ref)
            line += f" | v{v} max {(d.abs().max() / ref.abs().max()).item():.3e} rms {(d.norm() / ref.norm()).item():.3e}"
        K.wattn_fwd_policy(6, -2)
        print(line, flush=True)


if __name__ == "__main__":
    main()
