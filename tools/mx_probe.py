"""Decode the lane maps of the block-scaled MFMA from tools/mx_probe's hardware output.

    python tools/mx_probe.py gpurun_out/<dir>/mx_probe.bin

Prints, per shape, which output rows each A lane feeds, which columns each B lane feeds (under the standard
C/D layout of the shape), which B byte each A byte pairs with, which output entries a lane's E8M0 scale
governs, and an end-to-end check of the decoded model on random data; then checks v_cvt_pk_fp8_f32 against
torch's float -> float8_e4m3fn (round to nearest even).
"""
import sys

import numpy as np
import torch

NE = 386


def e4m3(b):
    return torch.from_numpy(np.array(b, dtype=np.uint8)).view(torch.float8_e4m3fn).float().numpy().astype(np.float64)


def cd(shape, D):
    """[64][16] lane/register output -> [M][M] matrix under the standard C/D layout."""
    M = 16 if shape == 16 else 32
    out = np.zeros((M, M))
    for l in range(64):
        if shape == 16:
            for r in range(4):
                out[4 * (l >> 4) + r, l & 15] = D[l, r]
        else:
            for r in range(16):
                out[(r & 3) + 8 * (r >> 2) + 4 * (l >> 5), l & 31] = D[l, r]
    return out


def kmap(shape, g, j):
    """Decoded operand map: byte j of lane group g (= lane // M) holds k = KH*(j >> 4) + 16 g + (j & 15), i.e. two
    16-byte halves, half h covering k in [KH h + 16 g, +16) with KH = 64 (16x16x128) or 32 (32x32x64)."""
    return (64 if shape == 16 else 32) * (j >> 4) + 16 * g + (j & 15)


def model(shape, a, b, sa, sb):
    """The decoded model: lane l holds A[row l%M][k = kmap(l // M, j)] in byte j (B: col); byte 0 of lane
    (i + M kb)'s scale VGPR is the E8M0 scale of row (col) i's k-block kb = k >> 5."""
    M = 16 if shape == 16 else 32
    fa = np.exp2((sa & 0xff).astype(np.float64) - 127)
    fb = np.exp2((sb & 0xff).astype(np.float64) - 127)
    R = np.zeros((M, M))
    for g in range(64 // M):
        for j in range(32):
            kb = kmap(shape, g, j) >> 5
            R += np.outer(a[g * M:(g + 1) * M, j] * fa[kb * M:(kb + 1) * M], b[g * M:(g + 1) * M, j] * fb[kb * M:(kb + 1) * M])
    return R


def main(path):
    raw = open(path, "rb").read()
    o = 0
    A = np.frombuffer(raw, np.uint8, NE * 2048, o).reshape(NE, 64, 32); o += NE * 2048
    B = np.frombuffer(raw, np.uint8, NE * 2048, o).reshape(NE, 64, 32); o += NE * 2048
    SA = np.frombuffer(raw, np.uint32, NE * 64, o).reshape(NE, 64); o += NE * 256
    SB = np.frombuffer(raw, np.uint32, NE * 64, o).reshape(NE, 64); o += NE * 256
    ok = True
    codes = e4m3(np.arange(0x38, 0x58))
    for shape in (16, 32):
        D = np.frombuffer(raw, np.float32, NE * 1024, o).reshape(NE, 64, 16); o += NE * 4096
        M = 16 if shape == 16 else 32
        print(f"=== {shape}x{shape}x{128 if shape == 16 else 64}")
        for L in (0, 1, 2, 3, 15, 16, 17, 31, 32, 33, 48, 63):
            m = cd(shape, D[L])
            rows = sorted(set(np.nonzero(m)[0]))
            mb = cd(shape, D[64 + L])
            cols = sorted(set(np.nonzero(mb)[1]))
            print(f"  A lane {L:2d} -> rows {rows} vals {sorted(set(m[m != 0]))};  B lane {L:2d} -> cols {cols} "
                  f"vals {sorted(set(mb[mb != 0]))}")
        for L in (0, 1, 16, 17, 32, 48):
            for e0, sv in ((128, 120), (192, 134)):
                m = cd(shape, D[e0 + L]) - (128 if shape == 16 else 64)
                print(f"  A scale lane {L:2d} = {sv}: changed rows {sorted(set(np.nonzero(m)[0]))} "
                      f"delta {sorted(set(m[m != 0]))}")
        base = cd(shape, D[256])
        for L in (0, 1, 16, 17, 32, 48):
            m = cd(shape, D[256 + L]) - (128 if shape == 16 else 64)
            mb = cd(shape, D[320 + L]) - (128 if shape == 16 else 64)
            print(f"  A scale lane {L:2d}: changed rows {sorted(set(np.nonzero(m)[0]))} delta {sorted(set(m[m != 0]))}; "
                  f"B scale lane {L:2d}: changed cols {sorted(set(np.nonzero(mb)[1]))} delta {sorted(set(mb[mb != 0]))}")
        del base
        for e in (384, 385):
            got = cd(shape, D[e])
            ref = model(shape, e4m3(A[e].reshape(-1)).reshape(64, 32), e4m3(B[e].reshape(-1)).reshape(64, 32),
                        SA[e], SB[e])
            err = np.abs(got - ref).max()
            print(f"  model check ({'A' if e == 384 else 'B'} scales random, decoded map): max |err| {err:.4g} of {np.abs(ref).max():.4g}")
            ok &= err == 0
    n = 1 << 16
    x = np.frombuffer(raw, np.float32, n, o); o += 4 * n
    y = np.frombuffer(raw, np.uint8, n, o)
    ref = torch.from_numpy(x.copy()).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    inr = np.abs(x) <= 448
    bad = (ref != y) & inr
    print(f"cvt_pk_fp8_f32: {inr.sum()} in-range values, {bad.sum()} differ from torch RNE")
    ok &= not bad.any()
    print("MX PROBE", "OK" if ok else "MISMATCH")


if __name__ == "__main__":
    main(sys.argv[1])
