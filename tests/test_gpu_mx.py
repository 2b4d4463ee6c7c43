"""MX-fp8 kernels (dfk_mx_quant, dfk_gemm_mx) against the CPU definition in tests/mx_ref.py.

Quantisation is bit-exact (values and scale bytes).  The GEMM multiplies exactly the dequantised operands, so it
is held to the fp32 product of the dequantised matrices within accumulation-order error (1e-4 of the entry's
|A||B| magnitude: the MFMA sums each 128-k tile internally; a lane-map or scale error is O(1) of it) — the fp8
error itself is the quantisation's, tested bit for bit."""
import pytest
import torch

import mx_ref

pytestmark = pytest.mark.gpu


def _rand(shape, seed, scale=1.0, dtype=torch.bfloat16):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(shape, generator=g) * scale
    # a few blocks spanning many octaves, a zero block and tiny values: every scale branch
    x.view(-1)[:32] *= 1e3
    x.view(-1)[32:64] = 0.0
    x.view(-1)[64:96] *= 1e-6
    return x.to(dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(1, 128), (77, 384), (300, 1024)])
def test_mx_quant_bit_exact(shape, dtype):
    from deepfake_amd import kernels as K
    x = _rand(shape, 1, dtype=dtype)
    m = K.mx_quant(x.cuda())
    q, s = mx_ref.quant(x)
    assert torch.equal(m.q.cpu(), q), "e4m3 values differ"
    assert torch.equal(m.s.cpu(), s), "E8M0 scales differ"


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(128, 5), (256, 130), (512, 64), (1024, 512), (384, 200)])
def test_mx_quant_transposed_bit_exact(shape, dtype):
    """x [R, C] -> the MX operand of x^T ([C, R], blocks along R): the dX GEMM's W^T."""
    from deepfake_amd import kernels as K
    x = _rand(shape, 2, dtype=dtype)
    m = K.mx_quant(x.cuda(), transpose=True)
    q, s = mx_ref.quant(x.t().contiguous())
    assert torch.equal(m.q.cpu(), q)
    assert torch.equal(m.s.cpu(), s)


def _check_gemm(M, N, Kd, seed, **epi):
    from deepfake_amd import kernels as K
    a = _rand((M, Kd), seed)
    b = _rand((N, Kd), seed + 1, scale=Kd ** -0.5)
    ma, mb = K.mx_quant(a.cuda()), K.mx_quant(b.cuda())
    A, B = mx_ref.dequant(ma.q.cpu(), ma.s.cpu()), mx_ref.dequant(mb.q.cpu(), mb.s.cpu())
    ref = (A.double() @ B.double().t())
    mag = (A.abs().double() @ B.abs().double().t())
    kw = {}
    if epi.get("bias"):
        bias = _rand((N,), seed + 2)
        kw["bias"] = bias.cuda()
        ref = ref + bias.double()
    if epi.get("gelu"):
        kw["act"], kw["aux"] = 1, torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    if epi.get("residual"):
        res = _rand((M, N), seed + 3)
        kw["residual"] = res.cuda()
    out = K.gemm_mx(ma, mb, **kw).float().cpu()
    # bf16 outputs: one rounding (2^-8 relative) on top of the accumulation-order error (1e-4 of |A||B|)
    if epi.get("gelu"):
        pre = ref
        aux = kw["aux"].float().cpu().double()
        assert bool(((aux - pre).abs() <= 1e-4 * mag + 2 ** -8 * pre.abs() + 1e-6).all())
        ref = torch.nn.functional.gelu(pre)
        mag = 1.2 * mag                      # |GELU'| <= 1.13 carries the accumulation error through
    if epi.get("residual"):
        ref = ref + res.double()
    tol = 1e-4 * mag + 2 ** -8 * ref.abs() + 2e-5 * ref.abs() + 1e-6
    err = (out.double() - ref).abs()
    assert bool((err <= tol).all()), float((err / tol).max())


@pytest.mark.parametrize("M,N,Kd", [(64, 64, 128), (100, 70, 256), (1568, 1536, 512), (2500, 640, 1024)])
def test_gemm_mx_plain(M, N, Kd):
    """Ragged M / N, both tile shapes (64x64 grids under 1024 128-tiles, 128x128 above)."""
    _check_gemm(M, N, Kd, 10)


def test_gemm_mx_large_tiles():
    _check_gemm(4096, 2048, 512, 20)


def test_gemm_mx_epilogues():
    """bias + GELU (pre-activation saved) and bias + residual: the dfk_gemm epilogues on the MX path."""
    _check_gemm(777, 512, 384, 30, bias=True, gelu=True)
    _check_gemm(640, 384, 512, 40, bias=True, residual=True)


def test_gemm_mx_rejects_bad_k():
    from deepfake_amd import kernels as K
    a = K.mx_quant(torch.randn(64, 256, device="cuda", dtype=torch.bfloat16))
    b = K.mx_quant(torch.randn(64, 128, device="cuda", dtype=torch.bfloat16))
    with pytest.raises(ValueError):
        K.gemm_mx(a, b)
    with pytest.raises(ValueError):
        K.mx_quant(torch.randn(64, 96, device="cuda", dtype=torch.bfloat16))


def test_gemm_mx_output_quantised_in_epilogue():
    """mx_out: the epilogue's MX copy of C equals dfk_mx_quant of the stored bf16 C, bit for bit (fc1 -> GELU -> the
    fc2 input, and the dGELU output feeding the fc1 dX GEMM)."""
    from deepfake_amd import kernels as K
    for M, N, Kd, act in ((333, 256, 128, 1), (2100, 1024, 256, 0)):
        a = _rand((M, Kd), 50).cuda()
        b = _rand((N, Kd), 51, scale=Kd ** -0.5).cuda()
        kw = {"act": 1, "aux": torch.empty(M, N, device="cuda", dtype=torch.bfloat16)} if act else {}
        out, mo = K.gemm_mx(K.mx_quant(a), K.mx_quant(b), bias=_rand((N,), 52).cuda(), mx_out=True, **kw)
        q, s = mx_ref.quant(out.float().cpu())
        assert torch.equal(mo.q.cpu(), q)
        assert torch.equal(mo.s.cpu(), s)
