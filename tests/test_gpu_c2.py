"""GPU parity at the headline configuration C2 (BASELINE.json configs[1]) against the reference's own
outputs (tests/golden/*.npz written by tests/golden/make_golden.py importing /root/reference):

* the stage-1 SW-MSA block over a whole clip's 16x56x56 volume (N=392 windows, shift 4x3x3: the launch
  the bench's roofline reports) and the stage-4 block whose only shift is along D (4,0,0; Q6);
* a SwinV2-B mel stage-3 block pair (14x14, C=512, 16 heads, shift 3, pretrained window 16);
* the whole fused model (Swin-T 32x224x224 + SwinV2-B mel + wav2vec2-base 4 s + FusionModel), B=2:
  eval logits, and one training forward+backward with EVERY parameter's gradient tensor compared
  (strided samples + norms);
* the fused C1 train step's gradient tensors (not only their norms).

Error = max|got - ref| / max|ref| per tensor (tests/fixtures.check).  Tolerances:
  fp32 parity mode (exact-fp32 MFMA): logits 1e-3 (the north-star bar), block outputs 1e-4, gradients 2e-3
  bf16 compute mode: eval logits 2e-2, train-mode logits (BatchNorm over 2 clips) 3e-2, block outputs 2e-2,
  block gradient tensors 5e-2; whole-model gradients: the relative L2 error of all gradients together
  <= 6e-2 and the median over tensors of (our error / the reference's own bf16 error) <= 1.5, with a
  per-tensor outlier guard max(1e-1, BF16_REF_FACTOR x the reference's own bf16 error on that tensor).
The last bound is measured, not chosen: make_golden.py runs the reference's step under torch.autocast(bf16)
too and stores each tensor's error against its fp32 run (``ea:<param>``; median 4.9 % at C1, 8.1 % at C2,
train logits 0.5 % / 5.4 %) — bf16 arithmetic alone puts most deep-layer gradients of this model above 5 %, so
a flat 5e-2 gate would fail every bf16 implementation, the reference's included.
A gradient whose reference is analytically zero (softmax shift invariance of the key biases) is checked
against an absolute floor instead (GRAD_FLOOR)."""
import numpy as np
import pytest
import torch

import golden_cases as GC
from fixtures import check, error, keys, load
from oracle.fill import named_fill_, randn, synthetic_inputs

pytestmark = pytest.mark.gpu
if torch.cuda.is_available():
    import deepfake_amd.models.swin_transformer2d as S2
    import deepfake_amd.models.video_swin_transformer as V
    from deepfake_amd.models.fused import build_fused

DEV = "cuda"
BLOCK_TOL = {torch.float32: (1e-4, 2e-4), torch.bfloat16: (2e-2, 5e-2)}
LOGIT_TOL = {torch.float32: 1e-3, torch.bfloat16: 2e-2}
GRAD_TOL = {torch.float32: 2e-3, torch.bfloat16: 5e-2}
GRAD_FLOOR = 1e-6   # |ref| below this (relative to the model's largest gradient) = analytically zero
BF16_REF_FACTOR = 6.0
TRAIN_LOGIT_TOL = {torch.float32: 1e-3, torch.bfloat16: 3e-2}


def _ref_scale(fx, k):
    return float(fx[k + "@norm"]) if k + "@norm" in fx else float(np.sqrt((fx[k].astype(np.float64) ** 2).sum()))


def check_grads(fx, named, tol, what="", ref_factor=None):
    """Every g:* tensor of the fixture against the model's .grad; returns the worst relative error.
    ref_factor: per-tensor bound max(tol, ref_factor * ea:<param>) (the reference's own bf16 error)."""
    ks = keys(fx, "g:")
    assert ks, "fixture holds no gradient tensors"
    top = max(_ref_scale(fx, k) for k in ks)
    errs = {}
    num = den = 0.0
    for k in ks:
        g = named[k[2:]].grad
        assert g is not None, f"{what}{k}: no gradient"
        if _ref_scale(fx, k) < GRAD_FLOOR * top:
            assert float(g.float().norm()) < 1e3 * GRAD_FLOOR * top, f"{what}{k}: should be ~0"
            continue
        errs[k[2:]] = error(fx, k, g)
        a = g.detach().double().cpu().reshape(-1).numpy()
        ref = fx[k + "@sub"] if k + "@sub" in fx else fx[k].reshape(-1)
        if k + "@sub" in fx:
            a = a[::int(fx[k + "@step"])]
        num += float(((a - ref) ** 2).sum())
        den += float((ref.astype(np.float64) ** 2).sum())
    l2 = (num / den) ** 0.5
    print(f"{what}relative L2 error of all gradients: {l2:.3e}")
    worst = sorted(errs.items(), key=lambda kv: -kv[1])
    print(f"{what}gradient tensors: {len(errs)} checked, worst {worst[:3]}, median {worst[len(worst) // 2]}")

    def bound(k):
        return max(2 * tol, ref_factor * float(fx["ea:" + k])) if ref_factor else tol
    if ref_factor:
        ratio = sorted(((k, e / max(float(fx["ea:" + k]), 1e-12)) for k, e in errs.items()), key=lambda kv: -kv[1])
        print(f"{what}error / reference-bf16 error: worst {ratio[:3]}, median {ratio[len(ratio) // 2]}")
        assert ratio[len(ratio) // 2][1] <= 1.5, f"{what}median error ratio to the reference's bf16 run > 1.5"
        # 6e-2: this build's bf16 gradients land 4.4e-2 .. 5.0e-2 from the fp32 reference (measured over
        # rounds 3-4), and the reference's own bf16 autocast run is at a median 8.1 % per tensor (ea:*).  It is
        # error, not run-to-run noise: two identical runs differ by 5.3e-8 relative L2 (forward, loss and logits
        # bitwise equal; only fp32 atomic order in weight-gradient sums moves, <= 3.5e-6 relative per tensor:
        # profiles/r5/r5a_determinism_c2_bf16.txt, tools/determinism_probe.py)
        assert l2 <= 6e-2, f"{what}relative L2 gradient error {l2:.3e}"
    bad = [(k, e, bound(k)) for k, e in worst if e > bound(k)]
    assert not bad, f"{what}{len(bad)} gradient tensors above {tol}: {bad[:8]}"
    return worst[0][1]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c", [GC.BLOCK_C2_S1, GC.BLOCK_C2_S4], ids=lambda c: c["name"])
def test_block_c2(dt, c):
    fx = load(c["name"])
    m = named_fill_(V.SwinTransformerBlock3D(c["dim"], c["heads"], window_size=tuple(c["window"]),
                                             shift_size=tuple(c["shift"])), c["seed"]).to(DEV)
    B, D, H, W = c["shape"]
    x = randn(c["seed"] + 1, (B, D, H, W, c["dim"])).to(DEV).to(dt).requires_grad_(True)
    y = m(x, None)
    y.backward(randn(c["seed"] + 2, y.shape).to(DEV).to(dt))
    tf, tb = BLOCK_TOL[dt]
    check(fx, "y", y, tf)
    check(fx, "dx", x.grad, tb)
    check_grads(fx, dict(m.named_parameters()), tb)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_mel_c2_stage3_pair(dt):
    c = GC.MEL_C2_S3
    fx = load(c["name"])
    m = S2.BasicLayer(dim=c["dim"], input_resolution=c["res"], depth=2, num_heads=c["heads"],
                      window_size=c["window"], pretrained_window_size=c["pretrained"])
    m = named_fill_(m, c["seed"]).to(DEV)
    H, W = c["res"]
    x = randn(c["seed"] + 1, (c["B"], H * W, c["dim"])).to(DEV).to(dt).requires_grad_(True)
    y = m(x)
    y.backward(randn(c["seed"] + 2, y.shape).to(DEV).to(dt))
    tf, tb = BLOCK_TOL[dt]
    check(fx, "y", y, tf)
    check(fx, "dx", x.grad, tb)
    check_grads(fx, dict(m.named_parameters()), tb)


def _fused(c, cfg_name, dt):
    m = named_fill_(build_fused(cfg_name, compute_dtype=dt), c["seed"]).to(DEV)
    video, mel, wave, label = synthetic_inputs(c["B"], c["T"], c["H"], c["W"], c["seconds"], seed=c["seed"] + 1)
    return m, (video.to(DEV), mel.to(DEV), wave.to(DEV)), label.to(DEV)


def _logit_err(z, ref):
    return float(np.abs(z - ref).max() / np.abs(ref).max())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fused_c2_eval_logits(dt):
    c = GC.FUSED_C2
    fx = load(c["name"])
    m, x, _ = _fused(c, "c2", dt)
    m.eval()
    with torch.no_grad():
        p = m(x)
    z = m.last_logits.float().cpu().numpy()
    err = _logit_err(z, fx["z_eval"])
    print(f"C2 eval logits rel err {err:.3e} ({dt}); reference's own bf16 autocast (train step): {float(fx['ea_logits']):.3e}")
    assert err < LOGIT_TOL[dt], (z, fx["z_eval"], err)
    assert np.abs(p.float().cpu().numpy() - fx["p_eval"]).max() < LOGIT_TOL[dt]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fused_c2_train_grads(dt):
    c = GC.FUSED_C2
    fx = load(c["name"])
    m, x, label = _fused(c, "c2", dt)
    m.train()
    p = m(x)
    loss = torch.nn.BCELoss()(p.float(), label)
    loss.backward()
    zerr = _logit_err(m.last_logits.float().cpu().numpy(), fx["z_train"])
    print(f"C2 train logits rel err {zerr:.3e} ({dt}); reference's own bf16 autocast {float(fx['ea_logits']):.3e}")
    assert zerr < TRAIN_LOGIT_TOL[dt]
    assert abs(loss.item() - float(fx["loss"])) < TRAIN_LOGIT_TOL[dt] * abs(float(fx["loss"]))
    check_grads(fx, dict(m.named_parameters()), GRAD_TOL[dt], what="c2 ",
                ref_factor=BF16_REF_FACTOR if dt == torch.bfloat16 else None)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fused_c1_grad_tensors(dt):
    c = GC.FUSED_C1
    fx = load("fused_c1_grads")
    m, x, label = _fused(c, "c1", dt)
    m.train()
    p = m(x)
    loss = torch.nn.BCELoss()(p.float(), label)
    loss.backward()
    assert abs(loss.item() - float(fx["loss"])) < LOGIT_TOL[dt] * abs(float(fx["loss"]))
    check_grads(fx, dict(m.named_parameters()), GRAD_TOL[dt], what="c1 ",
                ref_factor=BF16_REF_FACTOR if dt == torch.bfloat16 else None)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fused_c2_b8_eval_logits_vs_oracle(dt):
    """The bench's own batch (C2 at B = 8, the goldens hold B = 2): eval logits of the HIP path against the
    oracle (fp32 CPU restatement of the reference, pinned to the goldens) on the same weights and inputs —
    1e-3 relative in fp32 parity mode (the north-star bar), 2e-2 in bf16."""
    from deepfake_amd.models.fused import CONFIGS, W2V_CONFIG
    from oracle import fusion as OF
    cfg = CONFIGS["c2"]
    m = named_fill_(build_fused("c2", compute_dtype=dt), 21).to(DEV)
    ref = named_fill_(OF.build_fused(cfg, W2V_CONFIG), 21)
    video, mel, wave, _ = synthetic_inputs(8, cfg["T"], cfg["H"], cfg["W"], cfg["seconds"], seed=22)
    m.eval()
    ref.eval()
    with torch.no_grad():
        m((video.to(DEV), mel.to(DEV), wave.to(DEV)))
        ref((video, mel, wave))
    z, zr = m.last_logits.float().cpu().numpy(), ref.last_logits.numpy()
    err = _logit_err(z, zr)
    print(f"C2 B=8 eval logits rel err vs oracle {err:.3e} ({dt})")
    assert z.shape == zr.shape and err < LOGIT_TOL[dt], (z, zr, err)
