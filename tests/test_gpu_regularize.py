"""GPU: training-mode regularisers (dropout, DropPath, attention dropout, LayerDrop, SpecAugment).

Every mask is a counter-based hash evaluated inside the kernel that applies it (include/dfk.h dfk_drop,
deepfake_amd/rng.py).  The tests check (a) mask statistics against the reference's distributions
(nn.Dropout / timm DropPath: Bernoulli(1-p) scaled 1/(1-p); HF _compute_mask_indices span counts),
(b) that every fused site applies exactly the mask dfk_dropout reproduces (so forward and backward
agree), by comparing the fused kernels with plain torch fp32 references that use that mask, and (c)
that the masks change with the step counter and not with anything else.  Seeded: statistics are checked
with bounds several standard deviations wide.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from deepfake_amd import functional as Fn
    from deepfake_amd import kernels as K
    from deepfake_amd import rng

DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12)).item()


def mask_of(spec, rows, cols, dtype=torch.float32):
    """The mask a spec applies to a [rows, cols] output: dfk_dropout of ones (= keep / (1-p) or 0)."""
    return K.dropout(torch.ones(rows, cols, device=DEV, dtype=dtype), spec)


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_dropout_statistics_and_step(p):
    d = rng.Drop(p)
    m = mask_of(d.spec(), 2048, 768)
    keep = (m != 0).float()
    frac = 1 - keep.mean().item()
    n = m.numel()
    assert abs(frac - p) < 6 * math.sqrt(p * (1 - p) / n)
    assert torch.allclose(m[m != 0], torch.full_like(m[m != 0], 1 / (1 - p)))
    assert torch.equal(m, mask_of(d.spec(), 2048, 768))                  # same step: same mask
    rng.advance(DEV)
    m2 = mask_of(d.spec(), 2048, 768)
    assert not torch.equal(m, m2)                                        # next step: new mask
    assert abs((m2 != 0).float().mean().item() - (1 - p)) < 6 * math.sqrt(p * (1 - p) / n)
    other = mask_of(rng.Drop(p).spec(), 2048, 768)                        # another site: independent
    agree = ((other != 0) == (m2 != 0)).float().mean().item()
    assert abs(agree - (p * p + (1 - p) ** 2)) < 0.01
    # columns and rows are not correlated: per-column keep rates all near 1-p
    col = (m2 != 0).float().mean(0)
    assert (col - (1 - p)).abs().max().item() < 6 * math.sqrt(p * (1 - p) / 2048)


def test_droppath_groups():
    d = rng.Drop(0.2, mode=2)
    rows_per = 392
    m = mask_of(d.spec(rows_per), 4000 * rows_per // 100, 96)
    g = m.view(-1, rows_per, 96)
    first = g[:, :1, :1]
    assert torch.equal(g, first.expand_as(g))                             # one draw per clip
    frac = (first == 0).float().mean().item()
    assert abs(frac - 0.2) < 6 * math.sqrt(0.2 * 0.8 / first.numel())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mode,M,N,Kd", [(1, 1000, 288, 96), (2, 20000, 96, 384), (1, 1592, 768, 3072),
                                         (2, 1568, 512, 2048)])
def test_linear_dropout_epilogue(dt, mode, M, N, Kd):
    """y = residual + drop(x W^T + b) on the tiled, split-K and weight-resident GEMMs; the backward mask."""
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(M, Kd, device=DEV, generator=g).to(dt)
    w = (torch.randn(N, Kd, device=DEV, generator=g) / math.sqrt(Kd)).to(dt)
    b = torch.randn(N, device=DEV, generator=g).to(dt)
    r = torch.randn(M, N, device=DEV, generator=g).to(dt)
    spec = rng.Drop(0.3, mode=mode).spec(M // 8 if mode == 2 else 1)
    y = K.linear(x, w, b, residual=r, drop=spec)
    m = mask_of(spec, M, N)
    ref = (x.float() @ w.float().t() + b.float()) * m + r.float()
    assert rel(y, ref) < (2e-2 if dt == torch.bfloat16 else 2e-5)
    # GELU + dropout (FFN activation dropout) and the dGELU backward with the same mask
    aux = torch.empty(M, N, device=DEV, dtype=dt)
    h = K.linear(x, w, b, act=1, aux=aux, drop=spec)
    pre = x.float() @ w.float().t() + b.float()
    assert rel(h, torch.nn.functional.gelu(pre) * m) < (2e-2 if dt == torch.bfloat16 else 2e-5)
    dy = torch.randn(M, Kd, device=DEV, generator=g).to(dt)
    w2 = (torch.randn(Kd, N, device=DEV, generator=g) / math.sqrt(N)).to(dt)
    dpre = K.linear_dx(dy, w2, act=2, aux=aux, drop=spec)
    pre_t = aux.float().requires_grad_(True)
    (torch.nn.functional.gelu(pre_t) * m * (dy.float() @ w2.float())).sum().backward()
    assert rel(dpre, pre_t.grad) < (3e-2 if dt == torch.bfloat16 else 1e-4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mode", [1, 2])
def test_layernorm_residual_dropout(dt, mode):
    """y = residual + drop(LN(x)) and its backward (SwinV2 post-norm DropPath; wav2vec2 LN -> dropout)."""
    rows, C = 3136, 256
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.randn(rows, C, device=DEV, generator=g).to(dt)
    res = torch.randn(rows, C, device=DEV, generator=g).to(dt)
    ln = torch.nn.LayerNorm(C).to(DEV)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    spec = rng.Drop(0.25, mode=mode).spec(196)
    xr = x.detach().clone().requires_grad_(True)
    rr = res.detach().clone().requires_grad_(True)
    y = Fn.LayerNormFn.apply(xr, ln.weight.to(dt), ln.bias.to(dt), 1e-5, rr, spec)
    m = mask_of(spec, rows, C)
    xf = x.float().requires_grad_(True)
    ref = res.float() + torch.nn.functional.layer_norm(xf, (C,), ln.weight, ln.bias) * m
    tol = 3e-2 if dt == torch.bfloat16 else 1e-5
    assert rel(y, ref) < tol
    dy = torch.randn(rows, C, device=DEV, generator=g).to(dt)
    y.backward(dy)
    ref.backward(dy.float())
    assert rel(xr.grad, xf.grad) < (5e-2 if dt == torch.bfloat16 else 1e-4)
    assert rel(rr.grad, dy) == 0.0


def _w2v_attention_ref(qkv, B, T, heads, hd, m):
    C = heads * hd
    q, k, v = (qkv.float()[:, i * C:(i + 1) * C].reshape(B, T, heads, hd).transpose(1, 2) for i in range(3))
    p = torch.softmax(q @ k.transpose(-1, -2) * hd ** -0.5, dim=-1)
    return ((p * m) @ v).transpose(1, 2).reshape(B * T, C)


@pytest.mark.parametrize("T,heads,hd", [(199, 12, 64), (49, 2, 64), (96, 3, 32),
                                        (499, 2, 64)])   # Np 512: backward in query chunks, dK / dV accumulated
def test_attention_dropout(T, heads, hd):
    """HF eager_attention_forward with attention dropout (:458): O = (softmax(QK^T s) * Z) V; the kernel's
    forward and all three input gradients against a torch fp32 reference using the kernel's own mask."""
    B = 4
    C = heads * hd
    g = torch.Generator(device=DEV).manual_seed(3)
    qkv = (torch.randn(B * T, 3 * C, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    spec = rng.Drop(0.1).spec()
    Np = -(-T // 32) * 32
    z = mask_of(spec, B * heads * Np, Np).view(B, heads, Np, Np)[:, :, :T, :T]
    geo = ((B, 1, 1, T), (1, 1, T), (1, 1, T), (0, 0, 0), heads, hd, hd ** -0.5)
    x = qkv.detach().clone().requires_grad_(True)
    o = Fn.window_attention(x, None, None, geo, drop=spec)
    xf = qkv.float().requires_grad_(True)
    ref = _w2v_attention_ref(xf, B, T, heads, hd, z)
    assert rel(o, ref) < 2e-2
    frac = (z == 0).float().mean().item()
    assert abs(frac - 0.1) < 0.02
    do = torch.randn(B * T, C, device=DEV, generator=g).to(torch.bfloat16)
    o.backward(do)
    ref.backward(do.float())
    for i in range(3):
        assert rel(x.grad[:, i * C:(i + 1) * C], xf.grad[:, i * C:(i + 1) * C]) < 4e-2, i
    # p = 0 spec leaves the attention untouched
    o0 = Fn.window_attention(qkv, None, None, geo, drop=rng.Drop(0.0).spec())
    o1 = Fn.window_attention(qkv, None, None, geo)
    assert torch.equal(o0, o1)


def test_spec_augment():
    """HF _compute_mask_indices at wav2vec2-base settings (mask_time_prob 0.05, length 10, min_masks 2):
    T = 199 -> 2 distinct span starts per clip, spans of 10 frames (they may overlap)."""
    B, T, C = 64, 199, 768
    g = torch.Generator(device=DEV).manual_seed(4)
    h = torch.randn(B, T, C, device=DEV, generator=g).to(torch.bfloat16)
    emb = torch.randn(C, device=DEV, generator=g).to(torch.bfloat16)
    spec = rng.Drop(0.0).spec()
    out, mask = K.spec_augment_fwd(h, emb, 0.05, 10, 2, spec)
    mk = mask.bool()
    counts = mk.sum(1)
    assert ((counts >= 10) & (counts <= 20)).all()
    assert (counts == 20).float().mean().item() > 0.8          # non-overlapping spans are the common case
    for b in range(B):
        idx = mk[b].nonzero().flatten().tolist()
        runs = 1 + sum(1 for i, j in zip(idx, idx[1:]) if j != i + 1)
        assert 1 <= runs <= 2
    assert torch.equal(out[mk], emb.expand(int(mk.sum()), C))
    assert torch.equal(out[~mk], h[~mk])
    starts = torch.cat([mk[:, :1].int(), (mk[:, 1:].int() - mk[:, :-1].int()).clamp_min(0)], 1).nonzero()[:, 1]
    assert starts.float().mean().item() == pytest.approx((T - 10) / 2, abs=25)   # uniform over [0, 190)
    # backward: masked frames get no gradient, the embedding gets their sum
    dy = torch.randn(B, T, C, device=DEV, generator=g).to(torch.bfloat16)
    de = torch.zeros(C, device=DEV)
    dx = K.spec_augment_bwd(dy, mask, de)
    assert torch.equal(dx[mk], torch.zeros_like(dx[mk]))
    assert torch.equal(dx[~mk], dy[~mk])
    assert rel(de, dy.float()[mk].sum(0)) < 1e-5
    rng.advance(DEV)
    _, mask2 = K.spec_augment_fwd(h, emb, 0.05, 10, 2, spec)
    assert not torch.equal(mask, mask2)


def test_layerdrop_flags_and_sgd_gate():
    d = rng.Drop(0.1, shared=True)
    flags = K.bernoulli_flags(d.spec(), 100000, DEV)
    assert abs((flags == 0).float().mean().item() - 0.1) < 0.006
    # the SGD gate: a gated span is left untouched (param and momentum) when its flag is 0
    n = 1024
    p = torch.randn(n, device=DEV)
    gr = torch.randn(n, device=DEV)
    buf = torch.zeros(n, device=DEV)
    p0 = p.clone()
    K.sgd_step(p, gr, buf, None, 0.1, 0.9, 0.05, True, gate=torch.zeros(1, device=DEV))
    assert torch.equal(p, p0) and torch.equal(buf, torch.zeros_like(buf))
    K.sgd_step(p, gr, buf, None, 0.1, 0.9, 0.05, True, gate=torch.ones(1, device=DEV))
    assert rel(p, p0 - 0.1 * (gr + 0.05 * p0)) < 1e-6


@pytest.mark.parametrize("kept", [0.0, 1.0])
def test_layer_select_matches_where(kept):
    """The fused LayerDrop select (wav2vec2 encoder: a dropped layer returns its input) against torch.where,
    forward and both gradients, for a kept and a dropped layer (device flag)."""
    from deepfake_amd import functional as Fn
    g = torch.Generator(device=DEV).manual_seed(3)
    y = torch.randn(1592, 768, device=DEV, generator=g).to(torch.bfloat16).requires_grad_(True)
    x = torch.randn(1592, 768, device=DEV, generator=g).to(torch.bfloat16).requires_grad_(True)
    keep = torch.full((1,), kept, device=DEV)
    dout = torch.randn(1592, 768, device=DEV, generator=g).to(torch.bfloat16)
    out = Fn.LayerSelectFn.apply(y, x, keep)
    out.backward(dout)
    gy, gx = y.grad.clone(), x.grad.clone()
    y.grad = x.grad = None
    ref = torch.where(keep[0] > 0, y, x)
    ref.backward(dout)
    assert torch.equal(out, ref)
    assert torch.equal(gy, y.grad) and torch.equal(gx, x.grad)


@pytest.mark.parametrize("world", [3, 4])
def test_sgd_data_parallel_fold(world):
    """The fused step consumes the all-reduced SUM: grad_scale = 1 / world replaces the averaging pass, and
    grad_bf16 reads the bf16 bucket copy in place of the fp32 buffer (ddp.GradBucketer.finish(fold=True)).
    Odd lengths cover the scalar tail."""
    for n in (1000, 1003):
        g = torch.Generator(device=DEV).manual_seed(n)
        p0 = torch.randn(n, device=DEV, generator=g)
        gsum = torch.randn(n, device=DEV, generator=g) * world
        for first in (True, False):
            b0 = torch.randn(n, device=DEV, generator=g)
            # fp32 sum in the gradient buffer
            p, buf = p0.clone(), b0.clone()
            K.sgd_step(p, gsum, buf, None, 0.1, 0.9, 0.05, first, grad_scale=1.0 / world)
            gm = gsum * (1.0 / world) + 0.05 * p0
            bref = gm if first else 0.9 * b0 + gm
            assert rel(buf, bref) < 1e-6 and rel(p, p0 - 0.1 * bref) < 1e-6
            # bf16 sum in the bucket copy (the fp32 buffer holds something else and must not be read)
            gb = gsum.to(torch.bfloat16)
            p, buf = p0.clone(), b0.clone()
            K.sgd_step(p, torch.full_like(gsum, float("nan")), buf, None, 0.1, 0.9, 0.05, first,
                       grad_scale=1.0 / world, grad_bf16=gb)
            gm = gb.float() * (1.0 / world) + 0.05 * p0
            bref = gm if first else 0.9 * b0 + gm
            assert rel(buf, bref) < 1e-6 and rel(p, p0 - 0.1 * bref) < 1e-6


@pytest.mark.parametrize("fold", [False, True])
def test_sgd_runs_one_launch_matches_per_run(fold):
    """dfk_sgd_step_runs (every run of the step in one launch, optim.FusedSGD's default) against one dfk_sgd_step
    per run, bit for bit: ragged run lengths (scalar tails, runs shorter than a workgroup), gaps between runs left
    untouched, a dropped (gate 0) and a kept (gate 1) LayerDrop run, first / later momentum, the bf16 shadow, and
    the data-parallel fold (1 / world, bf16 bucket gradient)."""
    g = torch.Generator(device=DEV).manual_seed(7)
    n = 60000
    p0, g0, b0 = (torch.randn(n, device=DEV, generator=g) for _ in range(3))
    gb = (g0 * 3).to(torch.bfloat16) if fold else None
    off, on = torch.zeros(1, device=DEV), torch.ones(1, device=DEV)
    runs = [(0, 5003, None, True), (5008, 5012, off, False), (5016, 30000, on, False), (30008, 30009, None, False),
            (30016, 59999, None, True)]
    scale = 1.0 / 3 if fold else 1.0
    pa, ba, sa = p0.clone(), b0.clone(), torch.zeros(n, device=DEV, dtype=torch.bfloat16)
    for s, e, gate, first in runs:
        K.sgd_step(pa[s:e], g0[s:e], ba[s:e], sa[s:e], 0.0, 0.9, 0.05, first, lr_dev=torch.full((1,), 0.1, device=DEV),
                   gate=gate, grad_scale=scale, grad_bf16=gb[s:e] if gb is not None else None)
    pb, bb, sb = p0.clone(), b0.clone(), torch.zeros(n, device=DEV, dtype=torch.bfloat16)
    K.sgd_step_runs(pb, g0, bb, sb, runs, 0.9, 0.05, torch.full((1,), 0.1, device=DEV), grad_scale=scale,
                    grad_bf16=gb)
    torch.cuda.synchronize()
    assert torch.equal(pa, pb) and torch.equal(ba, bb) and torch.equal(sa, sb)
    for s, e in ((5003, 5016), (30000, 30008), (30009, 30016), (59999, n)):   # dropped run and gaps: untouched
        assert torch.equal(pb[s:e], p0[s:e]) and torch.equal(bb[s:e], b0[s:e])
    assert not torch.equal(pb[5016:30000], p0[5016:30000])


def test_fused_c1_regularized_step():
    """The C1 fused model with the reference's regularisers trains (finite loss, gradients everywhere the
    reference has them), its masks change from step to step, and eval mode is the deterministic model."""
    from deepfake_amd.ddp import GradBucketer
    from deepfake_amd.models.fused import build_fused
    from deepfake_amd.optim import FusedSGD
    from deepfake_amd.params import ParamStore
    from deepfake_amd.trainer import TrainStep
    from oracle.fill import named_fill_, synthetic_inputs
    torch.manual_seed(0)
    m = named_fill_(build_fused("c1", compute_dtype=torch.bfloat16, regularize=True), 7).cuda()
    ref = named_fill_(build_fused("c1", compute_dtype=torch.bfloat16, regularize=False), 7).cuda()
    video, mel, wave, label = synthetic_inputs(2, 8, 112, 112, 1, seed=5)
    feat = (video.cuda(), mel.cuda(), wave.cuda())
    m.eval()
    ref.eval()
    with torch.no_grad():
        za = m.head(m.vExtract(feat[0]), m.aExtract(feat[1]), m.paExtract.wav_model(feat[2])["last_hidden_state"]
                    .float().mean(1))
        zb = ref.head(ref.vExtract(feat[0]), ref.aExtract(feat[1]), ref.paExtract.wav_model(feat[2])["last_hidden_state"]
                      .float().mean(1))
    assert rel(za, zb) < 1e-6         # eval: no regulariser is active in the trunks (Audio2D's is bypassed here)
    m.train()
    store = ParamStore(m, torch.bfloat16)
    step = TrainStep(m, store, FusedSGD(store, 1e-3, 0.9, 0.05), GradBucketer(store), graph=False)
    losses = []
    for _ in range(3):
        loss, prob = step(feat, label.cuda())
        losses.append(loss.item())
        assert torch.isfinite(store.flat).all()
    assert all(math.isfinite(v) for v in losses)
    assert len(set(losses)) == 3


def test_layerdrop_gate_is_or_over_accumulation_window():
    """Gradient accumulation with LayerDrop (reference defaults: --accum_step 4, layerdrop 0.1): torch's SGD
    steps a layer's parameters iff their accumulated .grad is not None, i.e. iff the layer ran in ANY micro-step
    of the window (src/trainer.py:280-297, HF :700-706).  The fused SGD's gate must be the OR of the coins, not
    the last micro-step's coin: a layer kept earlier but dropped last is still stepped with the accumulated
    gradient; a layer dropped in every micro-step is left untouched (parameters and momentum)."""
    from deepfake_amd.models import set_compute_dtype
    from deepfake_amd.models.fused import W2V_CONFIG
    from deepfake_amd.models.wav2vec2 import Wav2Vec2Config, Wav2Vec2Encoder
    from deepfake_amd.optim import FusedSGD
    from deepfake_amd.params import ParamStore
    torch.manual_seed(0)
    cfg = Wav2Vec2Config.from_json_file(W2V_CONFIG, num_hidden_layers=8).deterministic()
    cfg.layerdrop = 0.5
    enc = set_compute_dtype(Wav2Vec2Encoder(cfg), torch.float32).to(DEV).train()
    store = ParamStore(enc, torch.float32)
    opt = FusedSGD(store, 0.1, 0.9, 0.05)
    g = torch.Generator(device=DEV).manual_seed(3)
    h = torch.randn(2, 49, 768, device=DEV, generator=g)
    wy = torch.randn(2, 49, 768, device=DEV, generator=g)
    # the coins depend on the LayerDrop site id, i.e. on how many dropout sites earlier tests created: take the
    # first seed whose window has a layer kept in an earlier micro-step and dropped in the last one
    for seed in range(11, 43):
        rng.manual_seed(seed, 0)
        store.zero_grad()
        coins = []
        for _ in range(4):
            rng.advance(DEV)
            (enc(h).float() * wy).sum().backward()
            coins.append(enc.layer_keep.clone())
        c = torch.stack(coins)
        used = c.amax(0)
        if bool(((c[-1] == 0) & (used == 1)).any()):
            break
    else:
        pytest.fail("no seed in 11..42 exercises kept-then-dropped")
    assert torch.equal(enc.layer_used, used)
    p0, g0 = store.flat.clone(), store.grad.clone()
    opt.step()
    for i, layer in enumerate(enc.layers):
        for p in layer.parameters():
            s, e = store.span(store.index[id(p)])
            if used[i] == 0:
                assert torch.equal(store.flat[s:e], p0[s:e]) and torch.equal(opt.buf[s:e], torch.zeros_like(opt.buf[s:e]))
            else:
                want = p0[s:e] - 0.1 * (g0[s:e] + 0.05 * p0[s:e])
                assert rel(store.flat[s:e], want) < 1e-6, (i, rel(store.flat[s:e], want))
    store.zero_grad()
    assert torch.equal(enc.layer_used, torch.zeros_like(enc.layer_used))


def _vst_block_ref(ob, x, z, pd, da, do, dp1, dp2):
    """oracle/vst.py's Swin3D block (video_swin_transformer.py:142-173, 219-278) in fp32 with the kernels' own
    masks injected: z on the softmax probabilities [windows, heads, N, N] (attn_drop, :165), pd on the proj
    output (proj_drop, :171), da / do after the GELU and after fc2 (Mlp's nn.Dropout, src/utils.py:257-259), and
    dp1 / dp2 the two DropPath draws; every token-row mask is indexed by the token's row b*DHW + (d*H + h)*W + w."""
    import torch.nn.functional as F
    from oracle.vst import clamp_window, shift_mask, window_token_index

    B, D, H, W, C = x.shape
    att = ob.attn
    ws, ss = clamp_window((D, H, W), ob.window_size, ob.shift_size)
    xn = F.layer_norm(x, (C,), ob.norm1.weight, ob.norm1.bias)
    Dp, Hp, Wp = [-(-n // w) * w for n, w in zip((D, H, W), ws)]
    xn = F.pad(xn, (0, 0, 0, Wp - W, 0, Hp - H, 0, Dp - D))
    tok = window_token_index(Dp, Hp, Wp, ws).to(x.device)
    d, h, w = tok // (Hp * Wp), (tok // Wp) % Hp, tok % Wp
    src = (((d + ss[0]) % Dp) * Hp + (h + ss[1]) % Hp) * Wp + (w + ss[2]) % Wp
    flat = xn.reshape(B, Dp * Hp * Wp, C)
    win = flat[:, src.reshape(-1)].reshape(B * tok.shape[0], tok.shape[1], C)
    B_, N = win.shape[:2]
    nH, hd = att.num_heads, C // att.num_heads
    qkv = att.qkv(win).view(B_, N, 3, nH, hd)
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
    s = (q * hd ** -0.5) @ k.transpose(-1, -2)
    bias = att.relative_position_bias_table[att.relative_position_index[:N, :N].reshape(-1)]
    s = s + bias.view(N, N, nH).permute(2, 0, 1)[None]
    if any(t > 0 for t in ss):
        m = shift_mask(Dp, Hp, Wp, ws, ss).to(x.device)
        s = (s.view(B_ // m.shape[0], m.shape[0], nH, N, N) + m[None, :, None]).view(B_, nH, N, N)
    o = ((torch.softmax(s, dim=-1) * z) @ v).transpose(1, 2).reshape(B_, N, C)
    y = att.proj(o).reshape(B, -1, C)
    a = torch.zeros_like(flat).index_copy(1, src.reshape(-1), y).view(B, Dp, Hp, Wp, C)[:, :D, :H, :W]
    x1 = x + (a.reshape(-1, C) * pd * dp1).view(B, D, H, W, C)
    hmid = F.gelu(ob.mlp.fc1(F.layer_norm(x1, (C,), ob.norm2.weight, ob.norm2.bias))).reshape(-1, 4 * C) * da
    return x1 + (ob.mlp.fc2(hmid) * do * dp2).view(B, D, H, W, C)


@pytest.mark.parametrize("attn_drop,drop,drop_path", [(0.0, 0.0, 0.0), (0.15, 0.0, 0.0), (0.0, 0.1, 0.0), (0.0, 0.0, 0.2),
                                                     (0.15, 0.1, 0.2)])
def test_swin3d_block_dropouts(attn_drop, drop, drop_path):
    """SwinTransformerBlock3D with attn_drop, drop (proj_drop and both Mlp dropouts) and drop_path > 0 (one at a
    time, then all together), training mode, bf16: forward and every gradient against the fp32 reference block
    using the kernels' masks (the attention mask row of (window w, head h, query q) is ((b nW + w) heads + h) Np + q,
    key = column).  Eval mode ignores every dropout (equal to the same block built with p = 0)."""
    import oracle.vst as OV
    from oracle.fill import named_fill_, randn
    import deepfake_amd.models.video_swin_transformer as V

    C, heads, win, shift = 96, 3, (8, 7, 7), (4, 3, 3)
    B, D, H, W = 2, 8, 14, 14
    blk = named_fill_(V.SwinTransformerBlock3D(C, heads, window_size=win, shift_size=shift, drop=drop,
                                               attn_drop=attn_drop, drop_path=drop_path), 5).to(DEV)
    ob = named_fill_(OV.SwinTransformerBlock3D(C, heads, win, shift), 5).to(DEV)
    x = randn(6, (B, D, H, W, C)).to(DEV)
    blk.train()
    xb = x.to(torch.bfloat16).requires_grad_(True)
    y = blk(xb, None)
    rows, nW, N, Np = B * D * H * W, 4, 392, 416
    ones = lambda r, c: torch.ones(r, c, device=DEV)   # noqa: E731
    z = (mask_of(blk.attn.attn_drop.spec(), B * nW * heads * Np, Np) if attn_drop else ones(B * nW * heads * Np, Np))
    z = z.view(B * nW, heads, Np, Np)[:, :, :N, :N]
    pd = mask_of(blk.attn.proj_drop.spec(), rows, C) if drop else ones(rows, C)
    da = mask_of(blk.mlp.sites[0].spec(), rows, 4 * C) if drop else ones(rows, 4 * C)
    do = mask_of(blk.mlp.sites[1].spec(), rows, C) if drop else ones(rows, C)
    dp1 = mask_of(blk.dp[0].spec(D * H * W), rows, C) if drop_path else ones(rows, C)
    dp2 = mask_of(blk.dp[1].spec(D * H * W), rows, C) if drop_path else ones(rows, C)
    for mm, p in ((z, attn_drop), (pd, drop), (da, drop), (do, drop)):
        assert abs((mm == 0).float().mean().item() - p) < 0.02
    xf = xb.detach().float().requires_grad_(True)
    ref = _vst_block_ref(ob, xf, z, pd, da, do, dp1, dp2)
    ey = rel(y, ref)
    dy = randn(7, y.shape).to(DEV).to(torch.bfloat16)
    y.backward(dy)
    ref.backward(dy.float())
    ex = rel(xb.grad, xf.grad)
    ours = dict(blk.named_parameters())
    errs = {n: rel(ours[n].grad, p.grad) for n, p in ob.named_parameters()}
    worst = max(errs.values())
    print(f"dropout block ({attn_drop}, {drop}, {drop_path}): y {ey:.3e} dx {ex:.3e} parameter gradients "
          + " ".join(f"{n} {e:.2e}" for n, e in errs.items()))
    assert ey < 2e-2 and ex < 5e-2 and worst < 5e-2
    # eval: no dropout anywhere
    blk.eval()
    ref0 = named_fill_(V.SwinTransformerBlock3D(C, heads, window_size=win, shift_size=shift), 5).to(DEV).eval()
    with torch.no_grad():
        assert torch.equal(blk(x.to(torch.bfloat16), None), ref0(x.to(torch.bfloat16), None))
