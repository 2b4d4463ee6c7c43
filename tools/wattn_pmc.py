"""N launches of one window-attention forward shape, for rocprofv3 --pmc passes.

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES ... -- python3 tools/wattn_pmc.py [stage] [N] [fwd|bwd]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepfake_amd import kernels as K  # noqa: E402

STAGES = {1: ((8, 16, 56, 56), 3), 2: ((8, 16, 28, 28), 6), 3: ((8, 16, 14, 14), 12), 4: ((8, 16, 7, 7), 24)}


def main():
    st = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    which = sys.argv[3] if len(sys.argv) > 3 else "fwd"
    dims, heads = STAGES[st]
    shift = (4, 3, 3) if st < 4 else (0, 0, 0)
    win = (8, 7, 7)
    hd, C = 32, heads * 32
    rows = dims[0] * dims[1] * dims[2] * dims[3]
    g = torch.Generator(device="cuda").manual_seed(7)
    qkv = torch.randn(rows, 3 * C, device="cuda", generator=g).to(torch.bfloat16)
    rpb = torch.randn(15 * 13 * 13, heads, device="cuda", generator=g) * 0.02
    args = (qkv, qkv[:, C:], qkv[:, 2 * C:], 3 * C, dims, win, win, shift, heads, hd, hd ** -0.5)
    out, lse, tab = K.wattn_fwd(*args, rpb=rpb, return_table=True)
    dout = torch.randn_like(out)
    dq = torch.empty_like(qkv)
    drpb = torch.zeros_like(rpb)
    for _ in range(n):
        if which == "fwd":
            K.wattn_fwd(*args, rpb=rpb, out=out)
        else:
            K.wattn_bwd(args[:4] and (qkv, qkv[:, C:], qkv[:, 2 * C:], out, lse, 3 * C, dims, win, win, shift, heads,
                                      hd, hd ** -0.5, rpb, None), dout, dq, dq[:, C:], dq[:, 2 * C:], 3 * C,
                        drpb=drpb, tab=tab)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
