"""Pin the CPU oracle to the reference's own outputs (golden fixtures generated
by importing /root/reference, tests/golden/make_golden.py).  CPU only."""

import pytest
import torch

import golden_cases as GC
from fixtures import check, keys, load
from oracle import fusion as OF
from oracle import swinv2 as S2
from oracle import vst as V
from oracle import w2v as W
from oracle.fill import named_fill_, randn, synthetic_inputs

RT = 2e-5  # fp32 restatement vs reference (different op order only)


def _grads(fx, m, rtol=RT):
    names = dict(m.named_parameters())
    ks = keys(fx, "g:")
    assert ks, "fixture has no grads"
    for k in ks:
        check(fx, k, names[k[2:]].grad, rtol)


@pytest.mark.parametrize("c", GC.WATTN_CASES, ids=lambda c: c["name"])
def test_window_attention(c):
    fx = load(c["name"])
    m = named_fill_(V.WindowAttention3D(c["dim"], c["full_window"], c["heads"]), c["seed"])
    x = randn(c["seed"] + 1, (c["B_"], c["N"], c["dim"])).requires_grad_(True)
    mask = None
    if c.get("mask_dhw"):
        # the fixture calls compute_mask with the raw (unclamped) window/shift
        mask = V.shift_mask(*c["mask_dhw"], c["full_window"], c["shift"])
    y = m(x, mask)
    y.backward(randn(c["seed"] + 2, y.shape))
    check(fx, "y", y, RT)
    check(fx, "dx", x.grad, RT)
    _grads(fx, m)


@pytest.mark.parametrize("c", GC.BLOCK_CASES + [GC.BLOCK_C4_S3], ids=lambda c: c["name"])
def test_block(c):
    fx = load(c["name"])
    m = named_fill_(V.SwinTransformerBlock3D(c["dim"], c["heads"], c["window"], c["shift"]), c["seed"])
    B, D, H, W_ = c["shape"]
    x = randn(c["seed"] + 1, (B, D, H, W_, c["dim"])).requires_grad_(True)
    y = m(x)
    y.backward(randn(c["seed"] + 2, y.shape))
    check(fx, "y", y, RT)
    check(fx, "dx", x.grad, RT)
    _grads(fx, m)


def test_patch_embed():
    c = GC.PATCH_EMBED
    fx = load(c["name"])
    m = named_fill_(V.PatchEmbed3D(c["patch"], 3, c["dim"]), c["seed"])
    y = m(randn(c["seed"] + 1, c["shape"]))
    y.backward(randn(c["seed"] + 2, y.shape))
    check(fx, "y", y, RT)
    _grads(fx, m)


@pytest.mark.parametrize("c", GC.MERGE_CASES, ids=lambda c: c["name"])
def test_patch_merging(c):
    fx = load(c["name"])
    m = named_fill_(V.PatchMerging(c["dim"]), c["seed"])
    x = randn(c["seed"] + 1, c["shape"]).requires_grad_(True)
    y = m(x)
    y.backward(randn(c["seed"] + 2, y.shape))
    check(fx, "y", y, RT)
    check(fx, "dx", x.grad, RT)
    _grads(fx, m)


def test_vst_c1():
    c = GC.VST_C1
    fx = load(c["name"])
    m = named_fill_(V.SwinTransformer3D(**c["kwargs"]), c["seed"])
    with torch.no_grad():
        y = m(randn(c["seed"] + 1, c["shape"]))
    check(fx, "y", y, 1e-4)


def test_w2v_2layer():
    c = GC.W2V_C1
    fx = load(c["name"])
    m = named_fill_(W.Wav2Vec2Model(W.W2VConfig(GC.W2V_CONFIG_JSON, num_hidden_layers=c["layers"])), c["seed"])
    _, _, wave, _ = synthetic_inputs(c["B"], 2, 16, 16, c["seconds"], seed=c["seed"] + 1)
    out = m(wave)
    h = out["last_hidden_state"]
    h.backward(randn(c["seed"] + 2, h.shape))
    check(fx, "y", h, 1e-4)
    check(fx, "extract", out["extract_features"], 1e-4)
    _grads(fx, m, 2e-4)


class _Ident(torch.nn.Module):
    def forward(self, x):
        return x


def test_fusion_head():
    c = GC.HEAD
    fx = load(c["name"])
    m = named_fill_(OF.FusionModel(_Ident(), _Ident(), _Ident(), 1, c["video_dim"], c["audio_dim"]), c["seed"])
    B = c["B"]
    fv = randn(c["seed"] + 1, (B, c["video_dim"])).requires_grad_(True)
    fa = randn(c["seed"] + 2, (B, c["audio_dim"])).requires_grad_(True)
    fp = randn(c["seed"] + 3, (B, 768)).requires_grad_(True)
    m.train()
    p = m((fv, fa, fp))
    check(fx, "z_train", m.last_logits, RT)
    p.backward(randn(c["seed"] + 4, p.shape))
    check(fx, "p_train", p, RT)
    for k, t in (("dfv", fv.grad), ("dfa", fa.grad), ("dfp", fp.grad), ("rm", m.norm.running_mean),
                 ("rv", m.norm.running_var)):
        check(fx, k, t, RT)
    _grads(fx, m)
    m.eval()
    with torch.no_grad():
        check(fx, "p_eval", m((fv, fa, fp)), RT)
        check(fx, "z_eval", m.last_logits, RT)


@pytest.mark.slow
def test_fused_c1_train_step():
    c = GC.FUSED_C1
    fx = load(c["name"])
    m = named_fill_(OF.build_fused(c, GC.W2V_CONFIG_JSON), c["seed"])
    video, mel, wave, label = synthetic_inputs(c["B"], c["T"], c["H"], c["W"], c["seconds"], seed=c["seed"] + 1)
    m.eval()
    with torch.no_grad():
        pe = m((video, mel, wave))
    check(fx, "p_eval", pe, 1e-4)
    check(fx, "z_eval", m.last_logits, 1e-4)
    m.train()
    opt = torch.optim.SGD(m.parameters(), lr=c["lr"], momentum=0.9, weight_decay=c["wd"])
    p = m((video, mel, wave))
    loss = torch.nn.BCELoss()(p, label)
    loss.backward()
    check(fx, "loss", loss, 1e-4)
    names = dict(m.named_parameters())
    bad = []
    for k in keys(fx, "gn:"):
        n = k[3:]
        g = names[n].grad
        ref = float(fx[k])
        if abs(float(g.norm()) - ref) > 1e-3 * ref + 1e-6:  # keys.bias grad is analytically 0
            bad.append((n, float(g.norm()), ref))
    assert not bad, bad[:5]
    opt.step()
    for k in keys(fx, "ps:"):
        n = k[3:]
        ref = float(fx[k])
        got = float(names[n].detach().double().sum())
        assert abs(got - ref) <= 1e-4 * max(1.0, abs(ref)), (n, got, ref)


def test_swinv2_masks_match_reference_construction():
    """The oracle's arithmetic mask equals compute-by-slices for a shifted 2D layer."""
    m = S2.shift_mask_2d(14, 14, 7, 3)
    assert m.shape == (4, 49, 49) and set(m.unique().tolist()) == {0.0, -100.0}

