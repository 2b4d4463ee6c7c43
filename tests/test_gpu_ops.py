"""GPU op-level numerics: each HIP kernel vs a plain PyTorch fp32 reference of the same op."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from deepfake_amd import kernels as K

DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12)).item()


def tol(dt):
    return 2e-2 if dt == torch.bfloat16 else 2e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,Kd", [(1000, 288, 96), (257, 96, 384), (64, 1536, 512), (3, 512, 1024),
                                    (1568, 512, 2048), (1592, 768, 3072),   # automatic split-K slabs
                                    (8200, 4104, 200)])   # 128x128 tiles, ragged M/N, K tail inside a k-tile
def test_linear_fwd_bwd(dt, M, N, Kd):
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(M, Kd, device=DEV, generator=g).to(dt)
    w = (torch.randn(N, Kd, device=DEV, generator=g) / math.sqrt(Kd)).to(dt)
    b = torch.randn(N, device=DEV, generator=g).to(dt)
    r = torch.randn(M, N, device=DEV, generator=g).to(dt)
    y = K.linear(x, w, b, residual=r)
    ref = x.float() @ w.float().t() + b.float() + r.float()
    assert rel(y, ref) < tol(dt)
    aux = torch.empty(M, N, device=DEV, dtype=dt)
    y2 = K.linear(x, w, b, act=1, aux=aux)
    pre = x.float() @ w.float().t() + b.float()
    assert rel(aux, pre) < tol(dt)
    assert rel(y2, torch.nn.functional.gelu(pre)) < tol(dt)
    dy = torch.randn(M, N, device=DEV, generator=g).to(dt)
    dx = K.linear_dx(dy, w)
    assert rel(dx, dy.float() @ w.float()) < tol(dt)
    dw = torch.zeros(N, Kd, device=DEV)
    K.linear_dw(dy, x, dw)
    assert rel(dw, dy.float().t() @ x.float()) < tol(dt)
    db = torch.zeros(N, device=DEV)
    K.colsum(dy, db)
    assert rel(db, dy.float().sum(0)) < tol(dt)
    # bias gradient fused into the dW pass (ones-operand MFMA)
    dw2 = torch.zeros(N, Kd, device=DEV)
    db2 = torch.zeros(N, device=DEV)
    K.linear_dw(dy, x, dw2, db=db2)
    assert rel(dw2, dy.float().t() @ x.float()) < tol(dt)
    assert rel(db2, dy.float().sum(0)) < tol(dt)


@pytest.mark.parametrize("M,N,Kd", [(20000, 288, 96), (16500, 96, 384), (17000, 384, 96), (16385, 576, 192),
                                    (20000, 512, 128), (16400, 192, 768), (16384, 96, 288)])
def test_linear_weight_resident(M, N, Kd):
    """bf16 Linears with >= 16k tokens and a small weight run on the weight-resident streaming kernel
    (wres.hip): ragged last row tile, several / partial column slices, every epilogue (bias, GELU with
    the pre-activation saved, dGELU, residual) and the transposed-weight dX form."""
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.randn(M, Kd, device=DEV, generator=g).to(dt)
    w = (torch.randn(N, Kd, device=DEV, generator=g) / math.sqrt(Kd)).to(dt)
    b = torch.randn(N, device=DEV, generator=g).to(dt)
    r = torch.randn(M, N, device=DEV, generator=g).to(dt)
    pre = x.float() @ w.float().t() + b.float()
    assert rel(K.linear(x, w, b, residual=r), pre + r.float()) < tol(dt)
    aux = torch.empty(M, N, device=DEV, dtype=dt)
    y = K.linear(x, w, b, act=1, aux=aux)
    assert rel(aux, pre) < tol(dt)
    assert rel(y, torch.nn.functional.gelu(pre)) < tol(dt)
    dy = torch.randn(M, N, device=DEV, generator=g).to(dt)
    assert rel(K.linear_dx(dy, w), dy.float() @ w.float()) < tol(dt)
    # fc2-style dX with the GELU derivative of a saved pre-activation: (dy W) * gelu'(aux2)
    aux2 = torch.randn(M, Kd, device=DEV, generator=g).to(dt)
    ref2 = (dy.float() @ w.float()) * torch.func.grad(lambda t: torch.nn.functional.gelu(t).sum())(aux2.float())
    assert rel(K.linear_dx(dy, w, act=2, aux=aux2), ref2) < tol(dt)
    # absent bias (the bias tile in LDS is zero) into an output pre-filled with NaN (no epilogue reads it), GELU
    # with a residual, and dGELU with a residual (the skip-path gradient) — the RES / ACT template pairs
    nobias = x.float() @ w.float().t()
    out = torch.full((M, N), float("nan"), device=DEV, dtype=dt)
    assert rel(K.linear(x, w, None, out=out), nobias) < tol(dt)
    aux3 = torch.full((M, N), float("nan"), device=DEV, dtype=dt)
    y3 = K.linear(x, w, None, act=1, aux=aux3, residual=r)
    assert rel(aux3, nobias) < tol(dt)
    assert rel(y3, torch.nn.functional.gelu(nobias) + r.float()) < tol(dt)
    r2 = torch.randn(M, Kd, device=DEV, generator=g).to(dt)
    assert rel(K.linear_dx(dy, w, act=2, aux=aux2, residual=r2), ref2 + r2.float()) < tol(dt)


@pytest.mark.parametrize("M,N,Kd", [(20000, 288, 96), (16500, 96, 96), (17000, 384, 96), (16400, 96, 384),
                                    (16385, 576, 192), (16384, 192, 768), (20000, 384, 128), (20000, 512, 128),
                                    (16384, 128, 512), (16448, 128, 128), (16400, 384, 768)])
def test_linear_dw_token_streaming(M, N, Kd, monkeypatch):
    """bf16 weight gradients with >= 16k tokens and a small dW on the token-streaming kernel (wgrad.hip, opt-in
    DFK_WGRAD=1):
    every instantiated wave grid, row / column slices (the bias gradient counted once per row), a ragged token
    tail, accumulation into a non-zero dW, and an x that is a column view of a wider buffer (ld > Kd).
    fp32 accumulation of exact bf16 products: checked at 1e-4 of the largest entry."""
    monkeypatch.setenv("DFK_WGRAD", "1")
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(3)
    xb = torch.randn(M, Kd + 64, device=DEV, generator=g).to(dt)
    x = xb[:, 32:32 + Kd]
    dy = torch.randn(M, N, device=DEV, generator=g).to(dt)
    dw0 = torch.randn(N, Kd, device=DEV, generator=g)
    db0 = torch.randn(N, device=DEV, generator=g)
    dw, db = dw0.clone(), db0.clone()
    K.linear_dw(dy, x, dw, db=db)
    ref = dw0.double() + dy.double().t() @ x.double()
    assert rel(dw, ref) < 1e-4
    assert rel(db, db0.double() + dy.double().sum(0)) < 1e-4
    dw2 = torch.zeros(N, Kd, device=DEV)
    K.linear_dw(dy, x, dw2)
    assert rel(dw2, dy.double().t() @ x.double()) < 1e-4


@pytest.mark.parametrize("slab", [False, True])
@pytest.mark.parametrize("M,N,Kd", [(50176, 96, 96), (40000, 384, 96), (1568, 2048, 512), (1592, 768, 3072),
                                    (40000, 100, 96), (40000, 96, 100)])
def test_linear_dw_bias_partials(M, N, Kd, slab, monkeypatch):
    """The weight gradient with its fused bias gradient on every split path: >= 32 atomic splits (the stage-1
    shapes: per-split bias partials + rowsum_reduce_kernel), few atomic splits (bias atomics), unsplit, and the fp32
    split-slab path (kernels._DW_SLAB: slab_sum_f32_kernel, bias partials after the slab) — against fp64, into
    non-zero dW / db.  N or Kd not a multiple of 8 runs the register-staged kernel, which adds the bias gradient
    atomically and writes no partials: no partial reduce may run on that path."""
    monkeypatch.setattr(K, "_DW_SLAB", slab)
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(M, Kd, device=DEV, generator=g).to(torch.bfloat16)
    dy = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    dw0 = torch.randn(N, Kd, device=DEV, generator=g)
    db0 = torch.randn(N, device=DEV, generator=g)
    dw, db = dw0.clone(), db0.clone()
    K.linear_dw(dy, x, dw, db=db)
    assert rel(dw, dw0.double() + dy.double().t() @ x.double()) < 1e-4
    assert rel(db, db0.double() + dy.double().sum(0)) < 1e-4


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,Kd", [(1000, 288, 96), (1568, 512, 2048), (1592, 768, 3072), (1592, 2304, 768)])
def test_inlaunch_combine(dt, M, N, Kd, monkeypatch):
    """Opt-in in-launch combine (DFK_INLAUNCH_COMBINE=1: arrival tickets, the last split / block group sums the
    partials): split-K forward / dX / dW GEMMs and the LayerNorm dgamma/dbeta partials equal the default path's
    results (same split order: bit-identical GEMM outputs)."""
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(M, Kd, device=DEV, generator=g).to(dt)
    w = (torch.randn(N, Kd, device=DEV, generator=g) / math.sqrt(Kd)).to(dt)
    dy = torch.randn(M, N, device=DEV, generator=g).to(dt)
    ln = torch.nn.LayerNorm(Kd).to(DEV)
    mean = x.float().mean(1)
    rstd = (x.float().var(1, unbiased=False) + 1e-5).rsqrt()
    dyl = torch.randn(M, Kd, device=DEV, generator=g).to(dt)

    def run():
        dw = torch.zeros(N, Kd, device=DEV)
        K.linear_dw(dy, x, dw)
        lw, lb = torch.zeros(Kd, device=DEV), torch.zeros(Kd, device=DEV)
        dxl = K.layernorm_bwd(dyl, x, ln.weight.to(dt), mean, rstd, lw, lb, slab_partials=True)
        return K.linear(x, w), K.linear_dx(dy, w), dw, dxl, lw, lb
    base = run()
    monkeypatch.setenv("DFK_INLAUNCH_COMBINE", "1")
    got = run()
    for i, (a, b) in enumerate(zip(got, base)):
        if i < 4 and i != 2:
            assert torch.equal(a, b), i
        else:   # group sums (and the dW of a split 128x128 grid: K.linear_dw) added atomically: order differs
            assert rel(a, b) < 1e-5, i


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,C",[(1000, 96), (33, 768), (17, 3072), (5, 512), (1001, 192), (77, 384), (9, 128),
                                    (13, 1536), (3, 1024), (29, 256)])
def test_layernorm(dt, rows, C):
    g = torch.Generator(device=DEV).manual_seed(1)
    x = (torch.randn(rows, C, device=DEV, generator=g) * 2 + 0.5).to(dt)
    w = (1 + 0.1 * torch.randn(C, device=DEV, generator=g)).to(dt)
    b = (0.1 * torch.randn(C, device=DEV, generator=g)).to(dt)
    y, mean, rstd = K.layernorm_fwd(x, w, b)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = b.float().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(xr, (C,), wr, br, 1e-5)
    assert rel(y, ref) < tol(dt)
    dy = torch.randn(rows, C, device=DEV, generator=g).to(dt)
    ref.backward(dy.float())
    dw = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    dx = K.layernorm_bwd(dy, x, w, mean, rstd, dw, db, slab_partials=False)   # atomic dw/db
    assert rel(dx, xr.grad) < tol(dt) * 2
    assert rel(dw, wr.grad) < tol(dt)
    assert rel(db, br.grad) < tol(dt)
    # dw/db through per-workgroup partials + column sums instead of atomics; dx accumulated onto a
    # residual-path gradient already in the output
    dw2 = torch.zeros(C, device=DEV)
    db2 = torch.zeros(C, device=DEV)
    dres = torch.randn(rows, C, device=DEV, generator=g).to(dt)
    dx2 = dres.clone()
    K.layernorm_bwd(dy, x, w, mean, rstd, dw2, db2, dx=dx2, accumulate=True, slab_partials=True)
    assert rel(dw2, wr.grad) < tol(dt)
    assert rel(db2, br.grad) < tol(dt)
    assert rel(dx2, xr.grad + dres.float()) < tol(dt) * 2


@pytest.mark.parametrize("heads,clamped", [(4, False), (32, True)])
def test_cpb_bias_and_cosine_logit_scale(heads, clamped):
    """SwinV2 16*sigmoid(cpb_mlp(coords)) (swin_transformer2d.py:159-162) and the cosine prologue with
    exp(clamp(logit_scale, max=log 100)) (:154-157), forward and parameter gradients vs torch fp32."""
    from deepfake_amd import functional as Fn
    g = torch.Generator(device=DEV).manual_seed(11)
    L = 169
    coords = torch.randn(1, 13, 13, 2, device=DEV, generator=g)
    mlp = torch.nn.Sequential(torch.nn.Linear(2, 512), torch.nn.ReLU(), torch.nn.Linear(512, heads, bias=False)).to(DEV)
    ref = 16 * torch.sigmoid(mlp(coords).view(-1, heads))
    w1, b1, w2 = (p.detach().clone().requires_grad_(True) for p in (mlp[0].weight, mlp[0].bias, mlp[2].weight))
    out = Fn.CPBBiasFn.apply(coords, w1, b1, w2)
    assert rel(out, ref) < 1e-5
    dout = torch.randn(L, heads, device=DEV, generator=g)
    out.backward(dout)
    ref.backward(dout)
    assert rel(w1.grad, mlp[0].weight.grad) < 1e-4
    assert rel(b1.grad, mlp[0].bias.grad) < 1e-4
    assert rel(w2.grad, mlp[2].weight.grad) < 1e-4
    # cosine prologue: q' = normalize(q) * exp(min(logit, log 100)), k' = normalize(k), v' = v
    rows, hd = 300, 32
    C = heads * hd
    qkv = torch.randn(rows, 3 * C, device=DEV, generator=g)
    logit = (torch.rand(heads, 1, 1, device=DEV, generator=g) * 2 + (4.0 if clamped else 1.0)).requires_grad_(True)
    x = qkv.clone().requires_grad_(True)
    y = Fn.CosineQKFn.apply(x, logit, heads, hd, math.log(100.0))
    xr = qkv.clone().requires_grad_(True)
    lr = logit.detach().clone().requires_grad_(True)
    s = torch.clamp(lr, max=math.log(100.0)).exp().view(1, heads, 1)
    q, k, v = (xr[:, i * C:(i + 1) * C].view(rows, heads, hd) for i in range(3))
    qn = (torch.nn.functional.normalize(q, dim=-1) * s).reshape(rows, C)
    kn = torch.nn.functional.normalize(k, dim=-1).reshape(rows, C)
    yr = torch.cat((qn, kn, v.reshape(rows, C)), 1)
    assert rel(y, yr) < 1e-5
    dy = torch.randn(rows, 3 * C, device=DEV, generator=g)
    y.backward(dy)
    yr.backward(dy)
    assert rel(x.grad, xr.grad) < 1e-4
    assert rel(logit.grad, lr.grad) < 1e-4


def test_cpb_tables_batched():
    """Every SwinV2 block's CPB table in one launch each way (Fn.cpb_tables, dfk_cpb_bias_*_many): forward tables
    and every parameter gradient equal the per-block kernels' (same arithmetic per table), over blocks of
    different head counts and window sizes — including a block whose table gets no gradient."""
    from deepfake_amd import functional as Fn
    from deepfake_amd.models.swin_transformer2d import WindowAttention
    torch.manual_seed(5)
    attns = [WindowAttention(64, (7, 7), 4, pretrained_window_size=(16, 16)),
             WindowAttention(128, (7, 7), 8), WindowAttention(512, (5, 5), 16),
             WindowAttention(1024, (7, 7), 32, pretrained_window_size=(16, 16))]
    attns = [a.to(DEV) for a in attns]
    tabs = Fn.cpb_tables(attns)
    douts = [torch.randn_like(t) for t in tabs]
    sum((t * d).sum() for t, d in zip(tabs[:3], douts[:3])).backward()   # the 4th table: no gradient
    got = [[p.grad.clone() if p.grad is not None else torch.zeros_like(p)
            for p in (a.cpb_mlp[0].weight, a.cpb_mlp[0].bias, a.cpb_mlp[2].weight)] for a in attns]
    for a in attns:
        a.zero_grad(set_to_none=True)
    for i, a in enumerate(attns):
        t = a.bias_table()
        assert rel(tabs[i], t) < 1e-6, i
        if i < 3:
            (t * douts[i]).sum().backward()
        for gp, p in zip(got[i], (a.cpb_mlp[0].weight, a.cpb_mlp[0].bias, a.cpb_mlp[2].weight)):
            ref = p.grad if p.grad is not None else torch.zeros_like(p)
            assert rel(gp, ref) < 1e-5 if i < 3 else float(gp.abs().max()) == 0.0, i


@pytest.mark.parametrize("C", [96, 384])
def test_skip_gradient_fusion(C):
    """Skip forms of LayerNormFn / MlpFn (one backward pass adds the gradient the input receives along the
    block's residual): a pre-norm block  y = x + mlp(LN(x))  built from the skip alias, a SwinV2-style
    post-norm  y = LN2(mlp(x)) + x  through MlpFn's alias, and wav2vec2's  x + FF(x)  with the residual
    being the input, each against the same graph in fp32 torch."""
    from deepfake_amd import functional as Fn
    torch.manual_seed(3)
    M = 300
    ln = torch.nn.LayerNorm(C).to(DEV)
    fc1, fc2 = torch.nn.Linear(C, 4 * C).to(DEV), torch.nn.Linear(4 * C, C).to(DEV)
    with torch.no_grad():
        for p in (ln.weight, ln.bias):
            p.add_(torch.randn_like(p) * 0.1)
    x0 = torch.randn(M, C, device=DEV)
    g = torch.randn(M, C, device=DEV)

    def ref_mlp(t):
        return fc2(torch.nn.functional.gelu(fc1(t)))

    def grads(fn):
        x = x0.clone().requires_grad_(True)
        for p in (*ln.parameters(), *fc1.parameters(), *fc2.parameters()):
            p.grad = None
        (fn(x) * g).sum().backward()
        return [x.grad] + [p.grad.clone() if p.grad is not None else None for p in (ln.weight, ln.bias, fc1.weight, fc2.weight)]

    def pre_norm(x):
        xn, xs = Fn.layer_norm(x, ln, skip=True)
        return Fn.mlp(xn, fc1, fc2, residual=xs)

    def post_norm(x):
        m, xs = Fn.mlp(x, fc1, fc2, skip=True)
        return Fn.layer_norm(m, ln, residual=xs)

    def res_input(x):
        return Fn.mlp(x, fc1, fc2, residual=x)

    cases = [(pre_norm, lambda x: x + ref_mlp(ln(x))), (post_norm, lambda x: x + ln(ref_mlp(x))),
             (res_input, lambda x: x + ref_mlp(x))]
    for ours, ref in cases:
        for a, b in zip(grads(ours), grads(ref)):
            if b is None:
                continue
            assert a is not None
            assert rel(a, b) < 1e-4


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("groups,R,C", [(8, 784, 768), (3, 5, 100), (2, 37, 1536), (1, 1, 64)])
def test_rowmean(dt, groups, R, C):
    """dfk_rowmean (VSTFeat's mean over a clip's tokens, the Inception global average pool) against torch."""
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(groups * R, C, device=DEV, generator=g).to(dt)
    out = K.rowmean(x, groups)
    ref = x.float().view(groups, R, C).mean(1)
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("heads,clamped,H", [(4, False, 14), (8, True, 21)])
def test_cosine_attention_logit_scale_dscore(heads, clamped, H):
    """SwinV2 window attention (swin_transformer2d.py:140-179: cosine scores * exp(clamp(logit_scale)) + 16
    sigmoid CPB bias, softmax, @ v) in bf16: the logit_scale gradient taken inside the attention backward
    (dfk_wattn_bwd_args.dscore: sum dS * score in fp32 with the exact softmax-backward row constant) against fp64
    autograd on the same bf16 inputs, and against the q-hat . dq' fallback (dscore off), which it must not lose to.
    The sum cancels to a few % of its terms, so its error is the precision of the whole chain."""
    from deepfake_amd import functional as Fn
    g = torch.Generator(device=DEV).manual_seed(21 + heads)
    B, W, ws, hd = 2, H, 7, 32
    C = heads * hd
    rows = B * H * W
    qkv = torch.randn(rows, 3 * C, device=DEV, generator=g).to(torch.bfloat16)
    L = (2 * ws - 1) ** 2
    tab = (16 * torch.sigmoid(torch.randn(L, heads, device=DEV, generator=g))).contiguous()
    logit0 = torch.rand(heads, 1, 1, device=DEV, generator=g) * 2 + (4.0 if clamped else 1.5)
    dout = torch.randn(rows, C, device=DEV, generator=g).to(torch.bfloat16)
    geo = ((B, 1, H, W), (1, ws, ws), (1, ws, ws), (0, 0, 0), heads, hd, 1.0)
    max_log = math.log(100.0)

    def run(use_dscore):
        logit = logit0.clone().requires_grad_(True)
        x = qkv.clone().requires_grad_(True)
        dsc = torch.zeros(heads, device=DEV) if use_dscore else None
        y = Fn.CosineQKFn.apply(x, logit, heads, hd, max_log, dsc)
        out = Fn.window_attention(y, tab, None, geo, dscore=dsc)
        out.backward(dout)
        if dsc is not None:
            assert dsc.abs().max().item() == 0.0   # consumed and re-zeroed by the cosine backward
        return out.detach(), logit.grad.flatten(), x.grad

    # fp64 reference on the same bf16 inputs
    lr = logit0.double().clone().requires_grad_(True)
    xr = qkv.double().clone().requires_grad_(True)
    q, k, v = (xr[:, i * C:(i + 1) * C].view(B, H // ws, ws, W // ws, ws, heads, hd) for i in range(3))
    part = lambda t: t.permute(0, 1, 3, 5, 2, 4, 6).reshape(-1, heads, ws * ws, hd)
    q, k, v = part(q), part(k), part(v)
    s = torch.clamp(lr, max=max_log).exp()
    # the kernels round q' = normalize(q) s and k' = normalize(k) to bf16 (CosineQKFn's output): the same rounding
    # here, straight through (forward rounded, gradient of the unrounded map)
    st = lambda t: t + (t.to(torch.bfloat16).double() - t).detach()
    qn = st(torch.nn.functional.normalize(q, dim=-1) * s.view(1, heads, 1, 1))
    kn = st(torch.nn.functional.normalize(k, dim=-1))
    attn = qn @ kn.transpose(-1, -2)
    yy, xx = torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")
    pos = (yy * (2 * ws - 1) + xx).flatten().to(DEV)
    idx = pos[:, None] - pos[None, :] + (ws - 1) * (2 * ws - 1) + (ws - 1)
    # the kernels' bias tables hold bias * log2(e) in bf16 (wattn.hip, wattn_tab3_kernel): the same quantisation
    l2e = 1.0 / math.log(2.0)
    tq = (tab.double() * l2e).to(torch.bfloat16).double() / l2e
    attn = attn + tq[idx].permute(2, 0, 1).unsqueeze(0)
    o = torch.softmax(attn, -1) @ v
    o = o.view(B, H // ws, W // ws, heads, ws, ws, hd).permute(0, 1, 4, 2, 5, 3, 6).reshape(rows, C)
    o.backward(dout.double())
    ref = lr.grad.flatten()

    out_n, dl_n, dx_n = run(True)
    out_o, dl_o, dx_o = run(False)
    assert torch.equal(out_n, out_o)
    # the q / k / v gradients: the same arithmetic up to where the score's bias joins it (C input of the product,
    # or added after it on the dscore path: fp32 rounding of S)
    assert rel(dx_n, dx_o) < 1e-2
    assert rel(out_n, o) < 5e-2   # scores up to s = 100: the bf16 Q' = q' log2(e) and bias tables quantise them
    err_n = ((dl_n.double() - ref).abs() / ref.abs().clamp_min(1e-30)).max().item()
    err_o = ((dl_o.double() - ref).abs() / ref.abs().clamp_min(1e-30)).max().item()
    print(f"logit_scale grad rel err: dscore {err_n:.3e}, q-hat.dq' {err_o:.3e}")
    # both carry the kernels' bf16 rounding of Q' = q' log2(e) before the scores (a few % here, where the sum cancels)
    assert err_n < 5e-2
    assert err_n <= err_o * 1.5 + 1e-4
