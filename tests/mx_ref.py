"""CPU reference of the MX-fp8 (OCP microscaling, e4m3 + E8M0 per 32 elements) quantisation and GEMM of
include/dfk.h (dfk_mx_quant / dfk_gemm_mx) — test infrastructure only.

The reference has no fp8 path (its Linears are fp32 / autocast): this is the definition the HIP kernels are held
to bit for bit, built on torch's float -> float8_e4m3fn conversion (round to nearest even), which the hardware's
v_cvt_pk_fp8_f32 matches on every in-range input (profiles/fp8/r4_mx_lane_map_probe.txt).
"""
import torch


def scale_bytes(amax):
    """E8M0 byte per block: the smallest e with amax / 2^(e-127) <= 448; all-zero blocks 127; clamp [1, 253]."""
    bits = amax.float().contiguous().view(torch.int32)
    E = (bits >> 23) & 0xFF
    e = E - 8 + ((bits & 0x7FFFFF) > 0x600000).to(torch.int32)
    e = torch.where(amax == 0, torch.full_like(e, 127), e)
    return e.clamp(1, 253)


def quant(x):
    """x [R, K] (K % 128 == 0) -> (q uint8 [R, K], s int32 [K/128, R]) exactly as dfk_mx_quant(transpose=0)."""
    x = x.float()
    R, K = x.shape
    xb = x.reshape(R, K // 32, 32)
    e = scale_bytes(xb.abs().amax(-1))                                   # [R, K/32]
    inv = torch.pow(2.0, (127 - e).float())[..., None]
    q = (xb * inv).to(torch.float8_e4m3fn).view(torch.uint8).reshape(R, K)
    eb = e.reshape(R, K // 128, 4).to(torch.int64)
    dw = eb[..., 0] | (eb[..., 1] << 8) | (eb[..., 2] << 16) | (eb[..., 3] << 24)
    s = dw.t().contiguous()
    s = torch.where(s >= 2 ** 31, s - 2 ** 32, s).to(torch.int32)
    return q, s


def dequant(q, s):
    """(q [R, K], s [K/128, R]) -> fp32 [R, K]."""
    R, K = q.shape
    v = q.contiguous().view(torch.float8_e4m3fn).float()
    dw = s.to(torch.int64) & 0xFFFFFFFF                                 # [K/128, R]
    e = torch.stack([(dw >> (8 * j)) & 0xFF for j in range(4)], -1)     # [K/128, R, 4]
    e = e.permute(1, 0, 2).reshape(R, K // 32).float()
    return (v.reshape(R, K // 32, 32) * torch.pow(2.0, e - 127)[..., None]).reshape(R, K)


def fq(x):
    """Fake quantisation: x [R, K] (K % 128 == 0) through MX-fp8 and back (blocks of 32 along the last dim)."""
    return dequant(*quant(x))


class MXLinearFn(torch.autograd.Function):
    """fp32 emulation of what set_fp8 does to one Linear (deepfake_amd/functional.py LinearFn / MlpFn, mx=True):
    forward y = fq(x) fq(W)^T + b (MX blocks along the in-features), input gradient dx = fq(dy) fq(W^T)^T (blocks
    along the out-features: the dX GEMM's contraction), weight / bias gradients from the unquantised x and dy (the
    weight-gradient GEMMs stay bf16).  Used by make_golden.py to measure the error MX-fp8 alone costs the reference
    model (the ``ef8:<param>`` anchors of tests/test_gpu_c4.py)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        x2 = x.reshape(-1, x.shape[-1])
        y = fq(x2) @ fq(w).t()
        if b is not None:
            y = y + b
        return y.reshape(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = (fq(dy2) @ fq(w.t().contiguous()).t()).reshape(x.shape)
        dw = dy2.t() @ x2
        db = dy2.sum(0) if ctx.has_b else None
        return dx, dw, db
