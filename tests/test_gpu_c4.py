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
2 clips) and loss 6e-2 (measured 4.2e-2; the reference's own bf16 autocast: 5.4e-2).
Whole-model gradients are anchored to the reference itself: make_golden.py (case_fused_c2_fp8) runs the reference's
C2 training step in fp32 with the same 32 Linears on MX-fp8 operands emulated (tests/mx_ref.MXLinearFn) and stores
each gradient's error against the plain fp32 step (``ef8:<param>``, median 4.2 %, RPB tables 5-14 %) and the
relative L2 over all gradients (``ef8_l2`` = 6.0e-2).  Bounds: per tensor max(1e-1, 6 x the reference's own bf16
error ``ea``, 2 x ``ef8``) — no tensor worse than the bf16 gate or twice what MX-fp8 alone costs the reference —
and, over the video tensors whose ``ef8`` exceeds ``ea`` (where fp8 dominates), median(error / ef8) <= 1.5; the
relative L2 of all gradients <= 1e-1, below the anchored ef8_l2 + the bf16 test's 6e-2 (measured 8.0-8.7e-2).
fp32 / bf16 rows keep test_gpu_c2.py's bounds."""
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
FP8_GRAD_FLOOR = 1e-1        # = test_gpu_c2's per-tensor floor (2 x GRAD_TOL)
FP8_REF_FACTOR = 2.0         # x ef8:<param>, the reference's own MX-fp8 error


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
    """Relative L2 error of all gradients together (sampled as the fixtures store them), the per-tensor bound
    max(FP8_GRAD_FLOOR, BF16_REF_FACTOR x ea, FP8_REF_FACTOR x ef8) and the median ratio to ef8 (module doc)."""
    from fixtures import keys
    from test_gpu_c2 import GRAD_FLOOR, _ref_scale
    f8 = load("fused_c2_fp8")
    assert FP8_GRAD_L2 <= float(f8["ef8_l2"]) + 6e-2, "L2 bound above the anchored sum"
    num = den = 0.0
    bad, ratios = [], []
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
        ea, ef8 = float(fx["ea:" + k[2:]]), float(f8["ef8:" + k[2:]])
        if e > max(FP8_GRAD_FLOOR, BF16_REF_FACTOR * ea, FP8_REF_FACTOR * ef8):
            bad.append((k, e, ea, ef8))
        if k.startswith("g:vExtract.") and ef8 > ea:
            ratios.append((e / ef8, k))
    l2 = (num / den) ** 0.5
    ratios.sort()
    med = ratios[len(ratios) // 2][0]
    print(f"fp8 relative L2 error of all gradients {l2:.3e} (reference fp8 emulation {float(f8['ef8_l2']):.3e}); "
          f"error / ef8 over {len(ratios)} fp8-dominated video tensors: median {med:.2f}, worst {ratios[-3:]}; "
          f"outliers {bad[:5]}")
    assert l2 <= FP8_GRAD_L2
    assert med <= 1.5, med
    assert not bad


@pytest.mark.parametrize("mode", ["bf16", "fp8"])
def test_fused_c4_whole_model(mode):
    """The whole C4 model (Swin-B video 2,2,18,2 / dim 128 + SwinV2-B mel + wav2vec2-base, 32x224x224 + 4 s, B=2;
    video_swin_transformer.py:462-550): eval logits against the oracle (fp32 CPU restatement of the reference,
    pinned to the goldens) built at the C4 configuration on the same weights and inputs — bf16 within the C2 bf16
    logit bound, fp8 (stages 3-4 on MX-fp8) within FP8_LOGIT_TOL — then one training forward + backward: finite
    loss near the oracle's, and a finite, non-zero gradient on every parameter the reference trains."""
    from deepfake_amd.models.fused import CONFIGS, W2V_CONFIG, build_fused
    from oracle import fusion as OF
    from test_gpu_c2 import LOGIT_TOL
    cfg = CONFIGS["c4"]
    m = named_fill_(build_fused("c4", compute_dtype=torch.bfloat16, fp8=mode == "fp8"), 41).to(DEV)
    ref = named_fill_(OF.build_fused(cfg, W2V_CONFIG), 41)
    video, mel, wave, label = synthetic_inputs(2, cfg["T"], cfg["H"], cfg["W"], cfg["seconds"], seed=42)
    x = (video.to(DEV), mel.to(DEV), wave.to(DEV))
    m.eval()
    ref.eval()
    with torch.no_grad():
        m(x)
        ref((video, mel, wave))
    z, zr = m.last_logits.float().cpu().numpy(), ref.last_logits.numpy()
    err = _logit_err(z, zr)
    tol = FP8_LOGIT_TOL if mode == "fp8" else LOGIT_TOL[torch.bfloat16]
    print(f"C4 {mode} eval logits rel err vs oracle {err:.3e} (bound {tol})")
    assert z.shape == zr.shape and err < tol, (z, zr, err)
    m.train()
    ref.train()
    p = m(x)
    loss = torch.nn.BCELoss()(p.float(), label.to(DEV))
    loss.backward()
    with torch.no_grad():
        lr_ = torch.nn.BCELoss()(ref((video, mel, wave)).float(), label).item()
    print(f"C4 {mode} train loss {loss.item():.5f} vs oracle {lr_:.5f}")
    assert np.isfinite(loss.item()) and abs(loss.item() - lr_) < FP8_TRAIN_LOGIT_TOL * abs(lr_)
    nz = 0
    for n, q in m.named_parameters():
        if q.grad is None:      # parameters the reference never uses (Audio2D.classifier, Q10)
            continue
        g = q.grad.float()
        assert torch.isfinite(g).all(), n
        nz += int(g.abs().max().item() > 0)
    assert nz >= 0.95 * len(list(m.parameters())), nz
