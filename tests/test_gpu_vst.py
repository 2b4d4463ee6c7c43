"""GPU parity: deepfake_amd VST modules (HIP path) vs the reference's golden
vectors (tests/golden, produced by the reference on CPU) on identical
named-fill weights and seeded inputs.

Tolerances (max|err| / max|ref|): fp32 parity mode (exact-fp32 MFMA) 1e-4;
bf16 compute mode 3e-2 (forward) / 6e-2 (gradients)."""
import pytest
import torch

import golden_cases as GC
from fixtures import check, keys, load
from oracle.fill import named_fill_, randn

pytestmark = pytest.mark.gpu
if torch.cuda.is_available():
    import deepfake_amd.models.video_swin_transformer as V
    from deepfake_amd.models import set_compute_dtype

DEV = "cuda"
TOL = {torch.float32: (1e-4, 2e-4), torch.bfloat16: (3e-2, 6e-2)}


def grads(fx, m, tol):
    names = dict(m.named_parameters())
    for k in keys(fx, "g:"):
        check(fx, k, names[k[2:]].grad, tol, what=f"[{k}] ")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c", GC.WATTN_CASES, ids=lambda c: c["name"])
def test_window_attention(dt, c):
    fx = load(c["name"])
    m = named_fill_(V.WindowAttention3D(c["dim"], c["full_window"], c["heads"], qkv_bias=True), c["seed"]).to(DEV)
    x = randn(c["seed"] + 1, (c["B_"], c["N"], c["dim"])).to(DEV).to(dt).requires_grad_(True)
    mask = None
    if c.get("mask_dhw"):
        mask = V.compute_mask(*c["mask_dhw"], tuple(c["full_window"]), tuple(c["shift"]), torch.device(DEV))
    y = m(x, mask)
    y.backward(randn(c["seed"] + 2, y.shape).to(DEV).to(dt))
    tf, tb = TOL[dt]
    check(fx, "y", y, tf)
    check(fx, "dx", x.grad, tb)
    grads(fx, m, tb)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c", GC.BLOCK_CASES, ids=lambda c: c["name"])
def test_block(dt, c):
    fx = load(c["name"])
    m = named_fill_(V.SwinTransformerBlock3D(c["dim"], c["heads"], window_size=tuple(c["window"]),
                                             shift_size=tuple(c["shift"])), c["seed"]).to(DEV)
    B, D, H, W = c["shape"]
    x = randn(c["seed"] + 1, (B, D, H, W, c["dim"])).to(DEV).to(dt).requires_grad_(True)
    y = m(x, None)
    y.backward(randn(c["seed"] + 2, y.shape).to(DEV).to(dt))
    tf, tb = TOL[dt]
    check(fx, "y", y, tf)
    check(fx, "dx", x.grad, tb)
    grads(fx, m, tb)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_patch_embed(dt):
    c = GC.PATCH_EMBED
    fx = load(c["name"])
    m = named_fill_(V.PatchEmbed3D(tuple(c["patch"]), 3, c["dim"], norm_layer=torch.nn.LayerNorm), c["seed"]).to(DEV)
    set_compute_dtype(m, dt)
    y = m(randn(c["seed"] + 1, c["shape"]).to(DEV))
    y.backward(randn(c["seed"] + 2, y.shape).to(DEV).to(dt))
    tf, tb = TOL[dt]
    check(fx, "y", y, tf)
    grads(fx, m, tb)


@pytest.mark.parametrize("shape,layout,C", [((2, 3, 8, 32, 32), "bcthw", 96), ((1, 32, 3, 224, 224), "btchw", 96),
                                            ((1, 7, 3, 30, 44), "btchw", 128), ((1, 4, 3, 224, 224), "btchw", 128)])
def test_patch_embed_fused_matches_unfused(shape, layout, C):
    """The fused bf16 pad + Conv3d + LayerNorm kernel (dfk_patch_embed_fwd/bwd) against the three-pass
    path (im2col -> GEMM -> LN) on the same inputs: C2 clip geometry in place ([B,T,3,H,W]), padded T/H/W,
    Swin-B width.  Outputs and all four parameter gradients."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(*shape, generator=g).to(DEV)
    outs = []
    for fused in (True, False):
        m = named_fill_(V.PatchEmbed3D((2, 4, 4), 3, C, norm_layer=torch.nn.LayerNorm), 17).to(DEV)
        set_compute_dtype(m, torch.bfloat16)
        m.force_unfused = not fused
        assert m.fused_ok(x) == fused
        y = m.tokens(x, layout)
        y.backward(torch.randn(y.shape, generator=g.manual_seed(4)).to(DEV).to(y.dtype))
        outs.append((y.float(), [p.grad.clone() for p in m.parameters()]))
    (yf, gf), (yu, gu) = outs
    assert (yf - yu).abs().max() / yu.abs().max() < 2e-2
    for a, b in zip(gf, gu):
        assert (a - b).abs().max() / b.abs().max() < 3e-2


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c", GC.MERGE_CASES, ids=lambda c: c["name"])
def test_patch_merging(dt, c):
    fx = load(c["name"])
    m = named_fill_(V.PatchMerging(c["dim"]), c["seed"]).to(DEV)
    x = randn(c["seed"] + 1, c["shape"]).to(DEV).to(dt).requires_grad_(True)
    y = m(x)
    y.backward(randn(c["seed"] + 2, y.shape).to(DEV).to(dt))
    tf, tb = TOL[dt]
    check(fx, "y", y, tf)
    check(fx, "dx", x.grad, tb)
    grads(fx, m, tb)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_vst_c1_forward(dt):
    c = GC.VST_C1
    fx = load(c["name"])
    m = named_fill_(V.SwinTransformer3D(**c["kwargs"]), c["seed"]).to(DEV)
    set_compute_dtype(m, dt)
    with torch.no_grad():
        y = m(randn(c["seed"] + 1, c["shape"]).to(DEV))
    check(fx, "y", y, 1e-3 if dt == torch.float32 else 5e-2)
