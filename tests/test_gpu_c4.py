"""GPU parity of C4 (BASELINE.json configs[3]: Swin-B video trunk, "fp8 MFMA attention/QKV path") against the
reference's own outputs (tests/golden/block_c4_*.npz, written by make_golden.py importing /root/reference):

* Swin-B blocks at stage 1 (dim 128, 4 heads, N=392 windows of a whole clip's 16x56x56 volume, shift 4x3x3) and
  stage 3 (dim 512, 16 heads, 16x14x14) in fp32 parity mode, bf16, and fp8 — bf16 compute with the block's
  qkv / proj / fc1 / fc2 forward and input-gradient GEMMs on MX-fp8 operands (e4m3 + one E8M0 scale per 32
  elements, dfk_gemm_mx); the weight gradients stay bf16;
* the fused C2 model with its video trunk's stage-3/4 Linears on MX-fp8 (the C4 default, models.set_fp8) against
  the C2 fp32 goldens: eval logits and every parameter's gradient.

Error = max|got - ref| / max|ref| per tensor (tests/fixtures.check).  Stated fp8 bounds (FP8_*): block output
3e-2, block input / parameter gradients 1e-1 (each MX operand carries e4m3's 2^-4 relative rounding, and the
input gradient goes through two MX dX GEMMs; measured r4e: y 1.1-1.3e-2, dx 1.4e-2, worst parameter gradient
7.0e-2, against bf16's 5-6e-3); fused C2 eval logits 1e-2 (measured 1.4e-3), train-mode logits (BatchNorm over
2 clips) and loss 6e-2 (measured 4.2e-2; the reference's own bf16 autocast: 5.4e-2); whole-model gradients:
relative L2 of all gradients together <= 1e-1 (measured 8.0-8.7e-2) with a per-tensor guard max(3.5e-1, 6 x the
reference's own bf16 autocast error on that tensor) — the relative-position-bias tables, sums of dS over every
window, carry the largest max-relative error (0.23 and 0.26 on two attention-kernel builds).  fp32 / bf16 rows keep test_gpu_c2.py's bounds."""
import numpy as np
import pytest
import torch

import golden_cases as GC
from fixtures import check, error, load
from oracle.fill import named_fill_, randn, synthetic_inputs
from test_gpu_c2 import BF16_REF_FACTOR, BLOCK_TOL, _fused, _logit_err, check_grads

pytestmark = pytest.mark.gpu
if torch.cuda.is_available():
    import deepfake_amd.models.video_swin_transformer as V
    from deepfake_amd.models import set_fp8

DEV = "cuda"
FP8_BLOCK_TOL = (3e-2, 1e-1)
FP8_LOGIT_TOL = 1e-2          # eval
FP8_TRAIN_LOGIT_TOL = 6e-2    # train mode (BatchNorm over 2 clips) and the loss
FP8_GRAD_L2 = 1e-1
FP8_GRAD_TENSOR = 3.5e-1


@pytest.mark.parametrize("mode", ["fp32", "bf16", "fp8"])
@pytest.mark.parametrize("c", [GC.BLOCK_C4_S1, GC.BLOCK_C4_S3], ids=lambda c: c["name"])
def test_block_c4(mode, c):
    fx = load(c["name"])
    dt = torch.float32 if mode == "fp32" else torch.bfloat16
    m = named_fill_(V.SwinTransformerBlock3D(c["dim"], c["heads"], window_size=tuple(c["window"]),
                                             shift_size=tuple(c["shift"])), c["seed"]).to(DEV)
    m.mx = mode == "fp8"
    B, D, H, W = c["shape"]
    x = randn(c["seed"] + 1, (B, D, H, W, c["dim"])).to(DEV).to(dt).requires_grad_(True)
    y = m(x, None)
    y.backward(randn(c["seed"] + 2, y.shape).to(DEV).to(dt))
    tf, tb = FP8_BLOCK_TOL if mode == "fp8" else BLOCK_TOL[dt]
    ey = check(fx, "y", y, tf)
    ex = check(fx, "dx", x.grad, tb)
    worst = check_grads(fx, dict(m.named_parameters()), tb, what=f"{c['name']} {mode} ")
    print(f"{c['name']} {mode}: y {ey:.3e}, dx {ex:.3e}, worst parameter gradient {worst:.3e}")


def test_fp8_switches_only_the_requested_stages():
    """set_fp8 marks the blocks of the requested stages and nothing else (C4 default: stages 3 and 4)."""
    from deepfake_amd.models.fused import build_fused
    m = build_fused("c4", compute_dtype=torch.bfloat16, fp8=True)
    vst = m.vExtract.vst
    assert [all(b.mx for b in layer.blocks) for layer in vst.layers] == [False, False, True, True]
    assert set_fp8(m, (0,)) == 2 and vst.layers[0].blocks[0].mx and not vst.layers[2].blocks[0].mx


def _fused_fp8(c):
    m, x, label = _fused(c, "c2", torch.bfloat16)
    assert set_fp8(m, (2, 3)) == 8
    return m, x, label


def test_fused_c2_fp8_eval_logits():
    """C2 with its stage-3/4 video Linears on MX-fp8, against the fp32 goldens."""
    c = GC.FUSED_C2
    fx = load(c["name"])
    m, x, _ = _fused_fp8(c)
    m.eval()
    with torch.no_grad():
        m(x)
    err = _logit_err(m.last_logits.float().cpu().numpy(), fx["z_eval"])
    print(f"C2 fp8 eval logits rel err {err:.3e} (bound {FP8_LOGIT_TOL})")
    assert err < FP8_LOGIT_TOL


def test_fused_c2_fp8_train_grads():
    c = GC.FUSED_C2
    fx = load(c["name"])
    m, x, label = _fused_fp8(c)
    m.train()
    p = m(x)
    loss = torch.nn.BCELoss()(p.float(), label)
    loss.backward()
    zerr = _logit_err(m.last_logits.float().cpu().numpy(), fx["z_train"])
    print(f"C2 fp8 train logits rel err {zerr:.3e}")
    assert zerr < FP8_TRAIN_LOGIT_TOL
    assert abs(loss.item() - float(fx["loss"])) < FP8_TRAIN_LOGIT_TOL * abs(float(fx["loss"]))
    _check_l2(fx, dict(m.named_parameters()))


def _check_l2(fx, named):
    """Relative L2 error of all gradients together (sampled as the fixtures store them), and the per-tensor
    guard max(FP8_GRAD_TENSOR, BF16_REF_FACTOR x the reference's own bf16 error)."""
    from fixtures import keys
    from test_gpu_c2 import GRAD_FLOOR, _ref_scale
    num = den = 0.0
    bad = []
    ks = keys(fx, "g:")
    top = max(_ref_scale(fx, k) for k in ks)
    for k in ks:
        g = named[k[2:]].grad
        assert g is not None, k
        if _ref_scale(fx, k) < GRAD_FLOOR * top:   # analytically zero (softmax shift invariance)
            continue
        a = g.detach().double().cpu().reshape(-1).numpy()
        ref = fx[k + "@sub"] if k + "@sub" in fx else fx[k].reshape(-1)
        if k + "@sub" in fx:
            a = a[::int(fx[k + "@step"])]
        num += float(((a - ref) ** 2).sum())
        den += float((ref.astype(np.float64) ** 2).sum())
        e = error(fx, k, g)
        if e > max(FP8_GRAD_TENSOR, BF16_REF_FACTOR * float(fx["ea:" + k[2:]])):
            bad.append((k, e))
    l2 = (num / den) ** 0.5
    print(f"fp8 relative L2 error of all gradients {l2:.3e}; outliers {bad[:5]}")
    assert l2 <= FP8_GRAD_L2
    assert not bad
