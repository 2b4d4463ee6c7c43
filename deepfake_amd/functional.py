"""Autograd functions over the HIP kernels (no CPU fallback: inputs must be on
the HIP device).  Parameters stay fp32 (the reference's state_dict dtype);
compute runs in the activation dtype (fp32 parity mode or bf16): weights are
read through ``compute_weight`` (the bf16 shadow kept by
deepfake_amd.params.ParamStore, else a per-call cast) and every weight /
bias gradient is produced in fp32.
"""
import os

import torch

from . import kernels as K


def _orig(p):
    """The ParamStore parameter behind p: p itself, or — for the detached alias an activation-checkpoint
    recompute hands back from ctx.saved_tensors — the parameter with the same storage (params.PARAM_BY_PTR)."""
    if p is None or hasattr(p, "_dfk_store") or not isinstance(p, torch.Tensor):
        return p
    from .params import PARAM_BY_PTR
    q = PARAM_BY_PTR.get(p.data_ptr())
    return q if q is not None and q.shape == p.shape else p


def compute_weight(p, dtype):
    """Weight in the compute dtype: the parameter itself (fp32) or its bf16 shadow."""
    if p is None:
        return None
    p = _orig(p)
    if p.dtype == dtype:
        return p
    sh = getattr(p, "_dfk_shadow", None)
    if sh is not None and sh.dtype == dtype:
        return sh
    return p.detach().to(dtype)


def _f32_zeros(p):
    return torch.zeros(p.shape, device=p.device, dtype=torch.float32)


def _store(p):
    return getattr(_orig(p), "_dfk_store", None) if p is not None else None


_RECOMPUTING = [0]   # > 0 inside an activation-checkpoint recompute (the use was counted in the first forward)


def grad_use(ctx, idx, p):
    """Forward side of a direct-gradient parameter: count this use so that the
    last backward contribution (grad_done) is the one that reports p ready."""
    p = _orig(p)
    st = _store(p)
    if st is not None and ctx.needs_input_grad[idx] and not _RECOMPUTING[0]:
        st.uses[id(p)] = st.uses.get(id(p), 0) + 1


def grad_sink(p):
    """fp32 buffer a backward kernel accumulates parameter p's gradient into.
    With a ParamStore in direct mode this is p.grad itself (a view of the flat
    gradient buffer, zeroed once per step): the kernels' fp32 atomics add
    straight into it and autograd never runs a fill or AccumulateGrad add for p."""
    p = _orig(p)
    st = _store(p)
    if st is not None:
        if p.grad is None:
            st.rebind_grads()
        return p.grad
    return _f32_zeros(p)


def grad_done(p, g):
    """Value to return to autograd for p, after its kernels accumulated into g
    (None in direct mode: the gradient is already in p.grad)."""
    p = _orig(p)
    st = _store(p)
    if st is None:
        return g
    st.grad_ready(p)
    return None


def checkpoint(fn, *args):
    """torch.utils.checkpoint (non-reentrant) of a region of HIP ops — the reference's use_checkpoint
    (video_swin_transformer.py:267-276, swin_transformer2d.py:428-429): the region's activations are dropped
    after the forward and recomputed in the backward.  The recompute is marked so direct-gradient use
    counts stay one per forward use, and the counter-based dropout masks (deepfake_amd.rng) redraw exactly
    the forward's masks (same seed, step and site)."""
    import contextlib
    import torch.utils.checkpoint as cp

    @contextlib.contextmanager
    def recompute():
        _RECOMPUTING[0] += 1
        try:
            yield
        finally:
            _RECOMPUTING[0] -= 1
    return cp.checkpoint(fn, *args, use_reentrant=False,
                         context_fn=lambda: (contextlib.nullcontext(), recompute()))


def rows2d(x):
    return x.reshape(-1, x.shape[-1])


def mx_weight(p, transpose=False):
    """MX-fp8 operand of a Linear weight [N, K] from its fp32 master: along K (the forward's B operand) or, with
    transpose, W^T along N (the dX GEMM's B operand).  Quantised per call, so a replayed graph always reads the
    weights SGD just wrote."""
    return K.mx_quant(_orig(p).detach(), transpose=transpose)


def mx_ok(x, weight, mx):
    """The MX-fp8 path applies: requested, bf16 activations, K and N multiples of 128."""
    return bool(mx) and x.dtype == torch.bfloat16 and x.shape[-1] % 128 == 0 and weight.shape[0] % 128 == 0


class LinearFn(torch.autograd.Function):
    """y = drop(x W^T + b) (act 1: drop(gelu(.))) (+ residual).  nn.Linear / F.linear, with the
    dropout / DropPath that follows it in the reference (rng.Drop spec, applied before the residual add).
    mx: the forward and the input-gradient GEMMs run on MX-fp8 operands (dfk_gemm_mx; C4's fp8 path), the
    weight gradient stays bf16."""

    @staticmethod
    def forward(ctx, x, weight, bias, act, residual, drop=None, mx=False):
        dt = x.dtype
        b = compute_weight(bias, dt)
        aux = torch.empty(x.shape[0], weight.shape[0], device=x.device, dtype=dt) if act == 1 else None
        if mx:
            y = K.gemm_mx(K.mx_quant(x), mx_weight(weight), bias=b, act=act, aux=aux, residual=residual, drop=drop)
        else:
            y = K.linear(x, compute_weight(weight, dt), b, act=act, aux=aux, residual=residual, drop=drop)
        grad_use(ctx, 1, weight)
        grad_use(ctx, 2, bias)
        ctx.save_for_backward(x, weight, bias, aux)
        ctx.act, ctx.has_bias, ctx.has_res, ctx.drop, ctx.mx = act, bias is not None, residual is not None, drop, mx
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, aux = ctx.saved_tensors
        dy = dy.contiguous()
        dz = K.dropout(dy, ctx.drop) if ctx.drop is not None else dy
        dz = K.gelu_bwd(dz, aux) if ctx.act == 1 else dz
        dx = None
        if ctx.needs_input_grad[0]:
            if ctx.mx:
                dx = K.gemm_mx(K.mx_quant(dz), mx_weight(weight, transpose=True))
            else:
                dx = K.linear_dx(dz, compute_weight(weight, x.dtype))
        dw = db = None
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            db = grad_sink(bias) if want_b else None      # bias gradient fused into the dW pass
            dw = grad_done(weight, K.linear_dw(dz, x, grad_sink(weight), db=db))
        elif want_b:
            db = K.colsum(dz, grad_sink(bias))
        if want_b:
            db = grad_done(bias, db)
        return dx, dw, db, None, (dy if ctx.has_res else None), None, None


def linear(x, weight, bias=None, act=0, residual=None, drop=None, mx=False):
    shp = x.shape
    x2 = rows2d(x).contiguous()
    y = LinearFn.apply(x2, weight, bias, act, rows2d(residual).contiguous() if residual is not None else None, drop,
                       mx_ok(x2, weight, mx))
    return y.view(*shp[:-1], weight.shape[0])


class GroupLinearFn(torch.autograd.Function):
    """y = x W^T + b where W (and b) are ParamStore adjacency groups (several parameters back to back, b
    possibly with zero gaps): the GEMMs read the flat master / bf16 shadow views in place and the backward
    writes dW / db straight into the flat gradient view, then reports every member ready."""

    @staticmethod
    def forward(ctx, x, st, wspan, wshape, bspan, skip, *params):
        dt = x.dtype
        src = st.shadow if (dt == torch.bfloat16 and st.shadow is not None) else st.flat
        if src.dtype != dt:
            raise RuntimeError("GroupLinearFn: compute dtype has no flat view")
        W = src[wspan[0]:wspan[0] + wspan[1]].view(wshape)
        B = src[bspan[0]:bspan[0] + bspan[1]] if bspan is not None else None
        y = K.linear(x, W, B)
        for i, p in enumerate(params):
            grad_use(ctx, 6 + i, p)
        ctx.save_for_backward(x, *params)
        ctx.st, ctx.wspan, ctx.wshape, ctx.bspan, ctx.skip = st, wspan, wshape, bspan, skip
        if skip:
            return y, x.view_as(x)
        return y

    @staticmethod
    def backward(ctx, dy, dskip=None):
        x, *params = ctx.saved_tensors
        st, (wo, wn), wshape, bspan = ctx.st, ctx.wspan, ctx.wshape, ctx.bspan
        dy = dy.contiguous()
        src = st.shadow if (x.dtype == torch.bfloat16 and st.shadow is not None) else st.flat
        # the skip alias's gradient (the block's residual path) joins dx in the GEMM epilogue
        dx = K.linear_dx(dy, src[wo:wo + wn].view(wshape), residual=dskip if ctx.skip else None) \
            if ctx.needs_input_grad[0] else None
        if any(p.grad is None for p in params):
            st.rebind_grads()
        db = st.grad[bspan[0]:bspan[0] + bspan[1]] if bspan is not None else None
        K.linear_dw(dy, x, st.grad[wo:wo + wn].view(wshape), db=db)
        for p in params:
            grad_done(p, None)
        return (dx, None, None, None, None, None) + (None,) * len(params)


def linear_group(x, weights, biases=None, skip=False):
    """nn.Linear over concatenated parameters: W = cat(weights) [sum N_i, K], b = cat(biases) with int
    entries of `biases` standing for zero gaps (SwinV2's qkv bias = cat(q_bias, 0, v_bias),
    swin_transformer2d.py:151-153; wav2vec2's separate q/k/v projections, HF :495-498).  With a ParamStore
    that laid the groups out adjacently (module.flat_groups()) nothing is concatenated; otherwise the
    reference's torch.cat.  skip=True also returns an alias of x for the block's residual consumer (its
    gradient is added in the dX GEMM epilogue; on the torch.cat fallback the alias is x itself)."""
    shp = x.shape
    x2 = rows2d(x).contiguous()
    st = _store(weights[0])
    if st is not None:
        ws = st.group_span(list(weights))
        bs = st.group_span(list(biases)) if biases is not None else None
        if ws is not None and (biases is None or bs is not None):
            wshape = (sum(w.shape[0] for w in weights), weights[0].shape[1])
            ps = list(weights) + [b for b in (biases or []) if not isinstance(b, int)]
            out = GroupLinearFn.apply(x2, st, ws, wshape, bs, skip, *ps)
            if skip:
                return out[0].view(*shp[:-1], wshape[0]), out[1].view(shp)
            return out.view(*shp[:-1], wshape[0])
    W = torch.cat(list(weights)) if len(weights) > 1 else weights[0]
    b = None
    if biases is not None:
        b = torch.cat([torch.zeros(e, device=x.device, dtype=weights[0].dtype) if isinstance(e, int) else e
                       for e in biases])
    y = linear(x, W, b)
    return (y, x) if skip else y


def _skip_grad_buffer(dskip, like):
    """The skip path's gradient as the LN backward's addend (read only: it is often a view of a grad_output the
    caller still holds, e.g. the gradient passed to y.backward(dy) at a block's output)."""
    if dskip.dtype == like.dtype and dskip.is_contiguous() and dskip.numel() == like.numel():
        return dskip.view(like.shape)
    return dskip.to(like.dtype).contiguous().reshape(like.shape)


class MlpFn(torch.autograd.Function):
    """residual + drop_out(fc2(drop_act(gelu(fc1(x))))) — src/utils.py:242-260 Mlp / HF Wav2Vec2FeedForward
    (:551-573: activation dropout after the GELU, hidden dropout after fc2) fused with the block residual
    (video_swin_transformer.py:276: DropPath of the branch = drop_out in group mode).
    Skip forms (no autograd add of two gradients of one tensor): res_is_input — the residual IS x (wav2vec2's
    x + FF(x), HF :587): dx = dpre W1 + dy in one GEMM epilogue; skip — a second output aliasing x for the
    block's other consumer of x (SwinV2's post-norm residual): its gradient is added in the same epilogue."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, residual, drop_act=None, drop_out=None, res_is_input=False, skip=False,
                mx=False):
        dt = x.dtype
        B1, B2 = compute_weight(b1, dt), compute_weight(b2, dt)
        pre = torch.empty(x.shape[0], w1.shape[0], device=x.device, dtype=dt)
        if mx:   # MX-fp8 GEMMs; the fc1 epilogue also writes h quantised for fc2 (no separate pass)
            h, hq = K.gemm_mx(K.mx_quant(x), mx_weight(w1), bias=B1, act=1, aux=pre, drop=drop_act, mx_out=True)
            y = K.gemm_mx(hq, mx_weight(w2), bias=B2, residual=residual, drop=drop_out)
        else:
            h = K.linear(x, compute_weight(w1, dt), B1, act=1, aux=pre, drop=drop_act)
            y = K.linear(h, compute_weight(w2, dt), B2, residual=residual, drop=drop_out)
        for i, p in enumerate((w1, b1, w2, b2)):
            grad_use(ctx, 1 + i, p)
        ctx.save_for_backward(x, w1, b1, w2, b2, pre, h)
        ctx.has_res, ctx.drop_act, ctx.drop_out = residual is not None, drop_act, drop_out
        ctx.res_is_input, ctx.skip, ctx.mx = res_is_input, skip, mx
        if skip:
            return y, x.view_as(x)
        return y

    @staticmethod
    def backward(ctx, dy, dskip=None):
        x, w1, b1, w2, b2, pre, h = ctx.saved_tensors
        dy = dy.contiguous()
        dyr = dy
        if ctx.drop_out is not None:
            dy = K.dropout(dy, ctx.drop_out)
        dt = x.dtype
        extra = dyr if ctx.res_is_input else (dskip if ctx.skip else None)
        if ctx.mx:   # (dy W2).Z * gelu'(pre) with its MX copy from the same epilogue, then dpre W1 on MX operands
            dpre, dpreq = K.gemm_mx(K.mx_quant(dy), mx_weight(w2, transpose=True), act=2, aux=pre, drop=ctx.drop_act,
                                    mx_out=True)
            dx = K.gemm_mx(dpreq, mx_weight(w1, transpose=True),
                           residual=extra.contiguous() if extra is not None else None) \
                if ctx.needs_input_grad[0] else None
        else:
            dpre = K.linear_dx(dy, compute_weight(w2, dt), act=2, aux=pre, drop=ctx.drop_act)   # (dy W2).Z * gelu'(pre)
            dx = K.linear_dx(dpre, compute_weight(w1, dt), residual=extra) if ctx.needs_input_grad[0] else None
        db2 = grad_sink(b2)
        dw2 = grad_done(w2, K.linear_dw(dy, h, grad_sink(w2), db=db2))
        db2 = grad_done(b2, db2)
        db1 = grad_sink(b1)
        dw1 = grad_done(w1, K.linear_dw(dpre, x, grad_sink(w1), db=db1))
        db1 = grad_done(b1, db1)
        dres = dyr if (ctx.has_res and not ctx.res_is_input) else None
        return dx, dw1, db1, dw2, db2, dres, None, None, None, None, None


def mlp(x, fc1, fc2, residual=None, drop_act=None, drop_out=None, skip=False, mx=False):
    """Mlp(x) (+ residual).  skip=True also returns an alias of x for the block's other consumer of x, whose
    gradient then joins dx inside the fc1 dX GEMM.  mx: MX-fp8 forward / dX GEMMs (C4's fp8 path)."""
    shp = x.shape
    x2 = rows2d(x).contiguous()
    res_is_input = residual is not None and residual is x
    r2 = x2 if res_is_input else (rows2d(residual).contiguous() if residual is not None else None)
    mx = mx_ok(x2, fc1.weight, mx) and fc2.weight.shape[0] % 128 == 0
    out = MlpFn.apply(x2, fc1.weight, fc1.bias, fc2.weight, fc2.bias, r2, drop_act, drop_out, res_is_input, skip, mx)
    if skip:
        y, xs = out
        return y.view(*shp[:-1], fc2.weight.shape[0]), xs.view(shp)
    return out.view(*shp[:-1], fc2.weight.shape[0])


class LayerNormFn(torch.autograd.Function):
    """y = LN(x), or residual + drop(LN(x)) (SwinV2 post-norm x + DropPath(LN(a)), swin_transformer2d.py:301,304;
    wav2vec2 LN -> dropout, HF :691-692)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, residual=None, drop=None, skip=False):
        dt = x.dtype
        y, mean, rstd = K.layernorm_fwd(x, compute_weight(weight, dt), compute_weight(bias, dt), eps,
                                        residual=residual, drop=drop)
        grad_use(ctx, 1, weight)
        grad_use(ctx, 2, bias)
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.drop, ctx.has_res, ctx.skip = drop, residual is not None, skip
        if skip:
            return y, x.view_as(x)
        return y

    @staticmethod
    def backward(ctx, dy, dskip=None):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        dw, db = grad_sink(weight), grad_sink(bias)
        if ctx.skip and dskip is not None:   # dx = LN'(dy) + the skip path's gradient, in one pass
            dx = K.layernorm_bwd(dy, x, compute_weight(weight, x.dtype), mean, rstd, dw, db, drop=ctx.drop,
                                 addend=_skip_grad_buffer(dskip, x))
        else:
            dx = K.layernorm_bwd(dy, x, compute_weight(weight, x.dtype), mean, rstd, dw, db, drop=ctx.drop)
        return dx, grad_done(weight, dw), grad_done(bias, db), None, (dy if ctx.has_res else None), None, None


def layer_norm(x, ln, residual=None, drop=None, skip=False):
    """LN(x) (residual + drop(LN(x))).  skip=True also returns an alias of x for the block's residual add:
    the gradient arriving there is accumulated into the LN backward's dx instead of a separate add."""
    shp = x.shape
    out = LayerNormFn.apply(rows2d(x).contiguous(), ln.weight, ln.bias, ln.eps,
                            rows2d(residual).contiguous() if residual is not None else None, drop, skip)
    if skip:
        return out[0].view(shp), out[1].view(shp)
    return out.view(shp)


class WindowAttnFn(torch.autograd.Function):
    """Window attention core on a token-major qkv buffer [rows, 3C]
    (video_swin_transformer.py:148-170 + forward_part1's pad/roll/partition
    :224-252).  Inputs: qkv, rpb table [L,nH] (fp32 param or None), qkv bias
    [3C] (the padded positions' q/k/v, or None), explicit mask or None."""

    @staticmethod
    def forward(ctx, qkv, rpb, qkv_bias, mask, geo, drop=None, dscore=None):
        dims, window, full_window, shift, heads, hd, scale = geo
        C = heads * hd
        pads = None
        if qkv_bias is not None:
            bc = compute_weight(qkv_bias, qkv.dtype)
            pads = (bc[:C], bc[C:2 * C], bc[2 * C:])
        rpb_f = rpb.detach().float().contiguous() if rpb is not None else None
        out, lse, tab = K.wattn_fwd(qkv, qkv[:, C:], qkv[:, 2 * C:], qkv.stride(0), dims, window, full_window, shift,
                                    heads, hd, scale, rpb=rpb_f, pads=pads, mask=mask, return_table=True, drop=drop)
        ctx.tab = tab
        # a batched CPB table (Fn.cpb_tables) hands its slice of the shared gradient buffer to its first consumer
        # only: a second consumer of the same table gets a fresh gradient, which autograd adds out of place
        ctx.gview = rpb.__dict__.pop("_dfk_gview", None) if rpb is not None else None
        grad_use(ctx, 1, rpb)
        grad_use(ctx, 2, qkv_bias)
        ctx.save_for_backward(qkv, out, lse, rpb_f, mask, rpb, qkv_bias)
        ctx.pads, ctx.geo, ctx.drop, ctx.dscore = pads, geo, drop, dscore
        ctx.has_rpb, ctx.has_bias = rpb is not None, qkv_bias is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, rpb_f, mask, rpb, qkv_bias = ctx.saved_tensors
        dims, window, full_window, shift, heads, hd, scale = ctx.geo
        C = heads * hd
        dqkv = torch.empty_like(qkv)
        drpb = None
        if ctx.has_rpb:
            if ctx.gview is not None:      # a batched CPB table: its zeroed slice of the shared gradient buffer
                drpb = ctx.gview
            else:
                drpb = grad_sink(rpb) if rpb.dtype == torch.float32 and rpb.is_contiguous() else torch.zeros_like(rpb_f)
            ctx.gview = None
        dbias = grad_sink(qkv_bias) if ctx.has_bias else None
        dpads = [dbias[i * C:(i + 1) * C] for i in range(3)] if ctx.has_bias else None
        K.wattn_bwd((qkv, qkv[:, C:], qkv[:, 2 * C:], out, lse, qkv.stride(0), dims, window, full_window, shift, heads,
                     hd, scale, rpb_f, ctx.pads), dout.contiguous(), dqkv, dqkv[:, C:], dqkv[:, 2 * C:], qkv.stride(0),
                    drpb=drpb, dpads=dpads, mask=mask, tab=ctx.tab, drop=ctx.drop, dscore=ctx.dscore)
        ctx.tab = None
        if ctx.has_rpb:
            drpb = grad_done(rpb, drpb)
        if ctx.has_bias:
            dbias = grad_done(qkv_bias, dbias)
        return dqkv, drpb, dbias, None, None, None, None


def window_attention(qkv, rpb, qkv_bias, geo, mask=None, drop=None, dscore=None):
    """drop: attention-probability dropout (bf16 table path only).  dscore: [heads] fp32 buffer the backward adds
    sum dS * score into (SwinV2's logit_scale gradient, consumed and re-zeroed by CosineQKFn's backward; bf16
    table path without dropout only — see dscore_buffer)."""
    if drop is not None and qkv.dtype != torch.bfloat16:
        raise NotImplementedError("attention dropout runs in the bf16 table kernels only (fp32 parity mode: p = 0)")
    return WindowAttnFn.apply(qkv, rpb, qkv_bias, mask, geo, drop, dscore)


def dscore_buffer(owner, qkv, heads, drop):
    """The [heads] fp32 buffer through which the attention backward hands sum dS * score to CosineQKFn's backward
    (dfk_wattn_bwd_args.dscore), or None where the attention kernel cannot produce it (fp32 parity mode, attention
    dropout, the table path switched off): CosineQKFn then derives the logit_scale gradient from q-hat . dq'.
    Persistent per module (zeroed once; the consumer re-zeroes it), so a captured step holds no fill for it."""
    if qkv.dtype != torch.bfloat16 or drop is not None or os.environ.get("DFK_WATTN_TABLE", "1") == "0" \
            or os.environ.get("DFK_COS_DSCORE", "0") != "1":
        return None
    buf = getattr(owner, "_dfk_dscore", None)
    if buf is None or buf.device != qkv.device or buf.numel() != heads:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("dscore buffer created inside a graph capture (run one eager step first)")
        buf = torch.zeros(heads, device=qkv.device, dtype=torch.float32)
        owner._dfk_dscore = buf
    return buf


class DropoutFn(torch.autograd.Function):
    """nn.Dropout / DropPath as a standalone pass on a 2-D view: y = x * mask / (1 - p)."""

    @staticmethod
    def forward(ctx, x, drop):
        ctx.drop = drop
        return K.dropout(x, drop)

    @staticmethod
    def backward(ctx, dy):
        return K.dropout(dy.contiguous(), ctx.drop), None


class LayerSelectFn(torch.autograd.Function):
    """LayerDrop (HF wav2vec2 encoder :700-706): out = y when the layer's device coin kept it, else its input x —
    one select launch forward and one backward (torch.where took a compare, the select, two fills and two selects)."""

    @staticmethod
    def forward(ctx, y, x, keep):
        ctx.save_for_backward(keep)
        return K.layer_select(y.contiguous(), x.contiguous(), keep)

    @staticmethod
    def backward(ctx, g):
        (keep,) = ctx.saved_tensors
        gy, gx = K.layer_select_bwd(g.contiguous(), keep)
        return gy, gx, None


class SpecAugmentFn(torch.autograd.Function):
    """HF Wav2Vec2Model._mask_hidden_states time masking (:1272-1317): masked frames <- masked_spec_embed."""

    @staticmethod
    def forward(ctx, h, embed, mask_prob, mask_length, min_masks, drop):
        e = compute_weight(embed, h.dtype).contiguous()
        out, mask = K.spec_augment_fwd(h.contiguous(), e, mask_prob, mask_length, min_masks, drop)
        grad_use(ctx, 1, embed)
        ctx.save_for_backward(mask, embed)
        return out

    @staticmethod
    def backward(ctx, dy):
        mask, embed = ctx.saved_tensors
        de = grad_sink(embed)
        dx = K.spec_augment_bwd(dy.contiguous(), mask, de)
        return dx, grad_done(embed, de), None, None, None, None


class PatchMergeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dims):
        ctx.dims = dims
        return K.patch_merge(x, dims)

    @staticmethod
    def backward(ctx, dy):
        return K.patch_merge(dy.contiguous(), ctx.dims, reverse=True), None


class RowMeanFn(torch.autograd.Function):
    """[groups*R, C] -> [groups, C] fp32 mean (per-clip token pooling)."""

    @staticmethod
    def forward(ctx, x, groups):
        ctx.shape, ctx.groups, ctx.dtype = x.shape, groups, x.dtype
        return K.rowmean(x, groups)

    @staticmethod
    def backward(ctx, dy):
        rows, C = ctx.shape
        R = rows // ctx.groups
        dx = (dy / R).to(ctx.dtype)[:, None, :].expand(ctx.groups, R, C).reshape(rows, C)
        return dx, None


class W2VConv0Fn(torch.autograd.Function):
    """wav2vec2 conv layer 0: Conv1d(1->512,k10,s5) + GroupNorm(512,512) + GELU
    (HF modeling_wav2vec2.py:302-323) -> channels-last [B, T0, 512]."""

    @staticmethod
    def forward(ctx, wave, weight, gamma, beta, eps, dtype):
        w = weight.detach().float().reshape(512, 10).contiguous()
        out, stats = K.w2v_conv0_fwd(wave.float().contiguous(), w, gamma.detach().float(), beta.detach().float(), eps,
                                     dtype)
        for i, p in enumerate((weight, gamma, beta)):
            grad_use(ctx, 1 + i, p)
        ctx.save_for_backward(wave, w, weight, gamma, beta, stats)
        ctx.eps = eps
        return out

    @staticmethod
    def backward(ctx, dout):
        wave, w, weight, gamma, beta, stats = ctx.saved_tensors
        dw, dg, db = grad_sink(weight), grad_sink(gamma), grad_sink(beta)
        K.w2v_conv0_bwd(wave.float().contiguous(), w, gamma.detach().float(), beta.detach().float(), ctx.eps, stats,
                        dout.contiguous(), dw.view(512, 10), dg, db)
        return None, grad_done(weight, dw), grad_done(gamma, dg), grad_done(beta, db), None, None


class ConvGeluFn(torch.autograd.Function):
    """Channels-last Conv1d(Cin->Cout, k, stride s, no bias) + GELU as an
    implicit GEMM (HF modeling_wav2vec2.py:253-272, conv layers 1..6):
    y[b,t,co] = gelu(sum_{kk,ci} W[co,ci,kk] x[b, s*t+kk, ci])."""

    @staticmethod
    def forward(ctx, x, weight, stride):
        B, Tin, Cin = x.shape
        Cout, _, k = weight.shape
        Tout = (Tin - k) // stride + 1
        dt = x.dtype
        w2 = weight.detach().permute(0, 2, 1).reshape(Cout, k * Cin).to(dt).contiguous()
        y = torch.empty(B, Tout, Cout, device=x.device, dtype=dt)
        pre = torch.empty_like(y)
        K.gemm(x, Cin, False, w2, k * Cin, False, Tout, Cout, k * Cin, y, Cout, dtype=K.L.dt(x), act=1, aux=pre,
               ldaux=Cout, nz=(B, 1), a_bs=(Tin * Cin, 0), c_bs=(Tout * Cout, 0), a_conv=(Cin, stride, 0, Tin))
        ctx.save_for_backward(x, w2, pre)
        ctx.meta = (stride, k, Cin, Cout, Tin, Tout, weight.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w2, pre = ctx.saved_tensors
        stride, k, Cin, Cout, Tin, Tout, wshape = ctx.meta
        B = x.shape[0]
        dt = K.L.dt(x)
        dpre = K.gelu_bwd(dy.contiguous(), pre)
        dw2 = torch.zeros(Cout, k * Cin, device=x.device)
        tiles = -(-Cout // 128) * -(-(k * Cin) // 128)
        K.gemm(dpre, Cout, True, x, Cin, True, Cout, k * Cin, Tout, dw2, k * Cin, dtype=dt, c_f32=True, atomic=True,
               splitk=max(1, min(K.splitk_for(tiles * B, Tout, 128), 16)), nz=(B, 1), a_bs=(Tout * Cout, 0),
               b_bs=(Tin * Cin, 0), b_conv=(Cin, stride, 0, Tin))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.zeros(B, Tin, Cin, device=x.device, dtype=x.dtype)
            for kk in range(k):  # col2im: tap kk of output t lands on input row stride*t + kk
                K.gemm(dpre, Cout, False, w2[:, kk * Cin:], k * Cin, True, Tout, Cin, Cout, dx[:, kk:], stride * Cin,
                       dtype=dt, beta=1.0, nz=(B, 1), a_bs=(Tout * Cout, 0), c_bs=(Tin * Cin, 0))
        dw = dw2.view(Cout, k, Cin).permute(0, 2, 1)
        return dx, dw, None


def _posconv_gemm_fwd(x, w2, bias, groups, k):
    """y = x + gelu(conv(x) + b) as the implicit GEMM per (clip, group); returns (y, pre-activation)."""
    B, T, C = x.shape
    Cg = C // groups
    dt = x.dtype
    y = torch.empty_like(x)
    pre = torch.empty_like(x)
    K.gemm(x, C, False, w2, k * Cg, False, T, Cg, k * Cg, y, C, dtype=K.L.dt(x), bias=compute_weight(bias, dt),
           bias_bs1=Cg, act=1, aux=pre, ldaux=C, residual=x, ldr=C, nz=(B, groups), a_bs=(T * C, Cg),
           b_bs=(0, Cg * k * Cg), c_bs=(T * C, Cg), r_bs=(T * C, Cg), a_conv=(Cg, 1, k // 2, T))
    return y, pre


def _posconv_gemm_bwd(x, dy, pre, w3, bias, groups, k):
    """-> (dx, dw2 [C, k*Cg] fp32 in the forward operand's layout, bias's gradient for autograd (None when the
    ParamStore already holds it))."""
    B, T, C = x.shape
    Cg = C // groups
    dt = K.L.dt(x)
    dy = dy.contiguous()
    dpre = K.gelu_bwd(dy, pre)
    db = grad_done(bias, K.colsum(dpre.view(-1, C), grad_sink(bias)))
    dw2 = torch.zeros(C, k * Cg, device=x.device)
    K.gemm(dpre, C, True, x, C, True, Cg, k * Cg, T, dw2, k * Cg, dtype=dt, c_f32=True, atomic=True,
           splitk=2, nz=(B, groups), a_bs=(T * C, Cg), b_bs=(T * C, Cg), c_bs=(0, Cg * k * Cg),
           b_conv=(Cg, 1, k // 2, T))
    # dx = dy + transposed conv: kernel flipped, pad k/2-1  (W3[g*Cg+ci][u*Cg+co] = W[g*Cg+co][ci][k-1-u])
    dx = dy.clone()
    K.gemm(dpre, C, False, w3, k * Cg, False, T, Cg, k * Cg, dx, C, dtype=dt, beta=1.0, nz=(B, groups),
           a_bs=(T * C, Cg), b_bs=(0, Cg * k * Cg), c_bs=(T * C, Cg), a_conv=(Cg, 1, k // 2 - 1, T))
    return dx, dw2, db


class PosConvFn(torch.autograd.Function):
    """x + gelu(grouped Conv1d(C, C, k, pad k/2, groups G)(x) + b) with the last
    output frame dropped (HF modeling_wav2vec2.py:326-380,689-690); weight is
    the (weight-normed) conv weight [C, C/G, k].  Implicit GEMM per (clip, group)."""

    @staticmethod
    def forward(ctx, x, weight, bias, groups):
        C = x.shape[2]
        Cg = C // groups
        k = weight.shape[2]
        w2 = weight.detach().permute(0, 2, 1).reshape(C, k * Cg).to(x.dtype).contiguous()  # [co][kk*Cg+ci]
        y, pre = _posconv_gemm_fwd(x, w2, bias, groups, k)
        grad_use(ctx, 2, bias)
        ctx.save_for_backward(x, weight, bias, pre)
        ctx.groups = groups
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, pre = ctx.saved_tensors
        C, G = x.shape[2], ctx.groups
        Cg, k = C // G, weight.shape[2]
        w3 = weight.detach().view(G, Cg, Cg, k).flip(3).permute(0, 2, 3, 1).reshape(C, k * Cg).to(x.dtype).contiguous()
        dx, dw2, db = _posconv_gemm_bwd(x, dy, pre, w3, bias, G, k)
        return dx, dw2.view(C, k, Cg).permute(0, 2, 1), db, None


class PosConvWNFn(torch.autograd.Function):
    """PosConvFn with the weight norm inside (HF weight_norm(dim=2): w = g v / ||v||_(0,1),
    modeling_wav2vec2.py:336-350): dfk_posconv_wnorm_fwd writes w straight into the forward GEMM's operand and the
    input-gradient GEMM's flipped operand (no torch weight-norm ops, permutes or casts), dfk_posconv_wnorm_bwd turns
    the dW GEMM's output into the gradients of g and v."""

    @staticmethod
    def forward(ctx, x, g, v, bias, groups):
        C = x.shape[2]
        Cg = C // groups
        k = v.shape[2]
        if v.shape[0] != C or v.shape[1] != Cg or g.numel() != k:
            raise ValueError("PosConvWNFn: v must be [C, C/groups, k] and g [1, 1, k]")
        vv, gg = v.detach().float().contiguous(), g.detach().float().contiguous()
        norm = torch.empty(k, device=x.device)
        ws = torch.empty(C * k, device=x.device)
        w2 = torch.empty(C, k * Cg, device=x.device, dtype=x.dtype)
        w3 = torch.empty_like(w2)
        K.posconv_wnorm_fwd(vv, gg, C, Cg, k, norm, ws, w2, w3)
        y, pre = _posconv_gemm_fwd(x, w2, bias, groups, k)
        grad_use(ctx, 1, g)
        grad_use(ctx, 2, v)
        grad_use(ctx, 3, bias)
        ctx.save_for_backward(x, gg, vv, bias, pre, w3, norm, g, v)
        ctx.groups = groups
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gg, vv, bias, pre, w3, norm, g, v = ctx.saved_tensors
        C, G = x.shape[2], ctx.groups
        Cg, k = C // G, vv.shape[2]
        dx, dw2, db = _posconv_gemm_bwd(x, dy, pre, w3, bias, G, k)
        dv, dg = grad_sink(v), grad_sink(g)
        ws = torch.empty(C * k, device=x.device)
        K.posconv_wnorm_bwd(vv, gg, norm, dw2, C, Cg, k, ws, dv, dg)
        return dx, grad_done(g, dg), grad_done(v, dv), db, None


class CosineQKFn(torch.autograd.Function):
    """SwinV2 cosine attention prologue: [rows, 3C] -> (normalize(q)*scale[h], normalize(k), v) with
    scale = exp(clamp(logit_scale, max=max_log)) computed in the kernel from the fp32 parameter
    (swin_transformer2d.py:154-157); the logit_scale gradient is accumulated directly."""

    @staticmethod
    def forward(ctx, qkv, logit_scale, heads, hd, max_log, dscore=None):
        out = torch.empty_like(qkv)
        ls = logit_scale.detach()
        if ls.dtype != torch.float32 or not ls.is_contiguous():
            ls = ls.float().contiguous()
        K.L.check(K.L.lib().dfk_cosine_qk_fwd(K.L.ptr(qkv), K.L.ptr(out), K.L.ptr(ls), float(max_log), qkv.shape[0],
                                              heads, hd, K.L.dt(qkv), K.L.stream()), "cosine_qk_fwd")
        grad_use(ctx, 1, logit_scale)
        ctx.save_for_backward(qkv, ls, logit_scale)
        ctx.hd, ctx.max_log, ctx.dscore = hd, max_log, dscore
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, ls, logit_scale = ctx.saved_tensors
        heads = ls.numel()
        dqkv = torch.empty_like(qkv)
        dls = grad_sink(logit_scale) if logit_scale.dtype == torch.float32 else torch.zeros_like(ls)
        K.L.check(K.L.lib().dfk_cosine_qk_bwd(K.L.ptr(qkv), K.L.ptr(dout.contiguous()), K.L.ptr(dqkv), K.L.ptr(ls),
                                              float(ctx.max_log), K.L.ptr(dls), qkv.shape[0], heads, ctx.hd,
                                              K.L.dt(qkv), K.L.ptr(ctx.dscore) if ctx.dscore is not None else None,
                                              K.L.stream()), "cosine_qk_bwd")
        return dqkv, grad_done(logit_scale, dls.view_as(logit_scale)), None, None, None, None


class CPBBiasFn(torch.autograd.Function):
    """SwinV2 relative-position bias table 16*sigmoid(cpb_mlp(relative_coords_table)) -> [L, heads] fp32
    (swin_transformer2d.py:159-162) in one kernel each way (dfk_cpb_bias_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, coords, w1, b1, w2):
        L, heads, hidden = coords.numel() // 2, w2.shape[0], w2.shape[1]
        c = coords.detach().float().reshape(L, 2).contiguous()
        W1, B1, W2 = (t.detach().float().contiguous() for t in (w1, b1, w2))
        out = torch.empty(L, heads, device=coords.device, dtype=torch.float32)
        K.L.check(K.L.lib().dfk_cpb_bias_fwd(K.L.ptr(c), K.L.ptr(W1), K.L.ptr(B1), K.L.ptr(W2), K.L.ptr(out), L,
                                             hidden, heads, K.L.stream()), "cpb_bias_fwd")
        for i, p in enumerate((w1, b1, w2)):
            grad_use(ctx, 1 + i, p)
        ctx.save_for_backward(c, W1, B1, W2, out, w1, b1, w2)
        return out

    @staticmethod
    def backward(ctx, dout):
        c, W1, B1, W2, out, w1, b1, w2 = ctx.saved_tensors
        L, heads, hidden = out.shape[0], W2.shape[0], W2.shape[1]
        d1, db, d2 = grad_sink(w1), grad_sink(b1), grad_sink(w2)
        K.L.check(K.L.lib().dfk_cpb_bias_bwd(K.L.ptr(c), K.L.ptr(W1), K.L.ptr(B1), K.L.ptr(W2), K.L.ptr(out),
                                             K.L.ptr(dout.float().contiguous()), K.L.ptr(d1), K.L.ptr(db), K.L.ptr(d2),
                                             L, hidden, heads, K.L.stream()), "cpb_bias_bwd")
        return None, grad_done(w1, d1), grad_done(b1, db), grad_done(w2, d2)


_CPB_DESC = {}   # (pointers, dims) -> device descriptor array of dfk_cpb_bias_*_many (built once, replay-safe)
_CPB_PINNED = set()   # keys a graph capture read: a captured graph dereferences them at every replay


def _cpb_desc(rows, device):
    key = tuple(tuple(r) for r in rows) + (str(device),)
    d = _CPB_DESC.get(key)
    capturing = torch.cuda.is_current_stream_capturing()
    if d is None:
        if capturing:
            raise RuntimeError("cpb descriptor built inside a graph capture (run one eager step first)")
        d = torch.tensor([v for r in rows for v in r], dtype=torch.int64, device=device)
        if len(_CPB_DESC) > 64:   # modules without a ParamStore get fresh gradient buffers every call
            for k in [k for k in _CPB_DESC if k not in _CPB_PINNED]:
                del _CPB_DESC[k]
        _CPB_DESC[key] = d
    if capturing:
        _CPB_PINNED.add(key)
    return d


class CPBManyFn(torch.autograd.Function):
    """Every SwinV2 block's relative-position bias table 16*sigmoid(cpb_mlp(coords)) (swin_transformer2d.py:159-162)
    in ONE launch forward (dfk_cpb_bias_fwd_many) and one backward (dfk_cpb_bias_bwd_many) — the tables depend on
    parameters only, so the 24 blocks of SwinV2-B need not pay 24 launches each way.  Inputs: the coordinate tables,
    then (w1, b1, w2) of every block; outputs: the [L, heads] tables (views of one fp32 buffer)."""

    @staticmethod
    def forward(ctx, n, *ts):
        coords, params = ts[:n], ts[n:]
        cs = [c.detach().float().reshape(-1, 2).contiguous() for c in coords]
        ws = [p.detach().float().contiguous() for p in params]
        dims, off, fwd_rows = [], 0, []
        for i in range(n):
            w1, b1, w2 = ws[3 * i:3 * i + 3]
            L, heads, hidden = cs[i].shape[0], w2.shape[0], w2.shape[1]
            assert heads <= 32, heads
            dims.append((off, L, heads))
            base = [cs[i].data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr()]
            fwd_rows.append(base + [0, 0, 0, off, L, hidden, heads, 0])
            off += L * heads
        out = torch.empty(off, device=cs[0].device, dtype=torch.float32)
        maxL = max(d[1] for d in dims)
        K.L.check(K.L.lib().dfk_cpb_bias_fwd_many(K.L.ptr(_cpb_desc(fwd_rows, out.device)), n, maxL, K.L.ptr(out),
                                                   K.L.stream()), "cpb_bias_fwd_many")
        for i, p in enumerate(params):
            grad_use(ctx, 1 + n + i, p)
        ctx.n, ctx.dims, ctx.maxL, ctx.fwd_rows = n, dims, maxL, fwd_rows
        ctx.save_for_backward(out, *cs, *ws, *params)   # cs / ws: the descriptor's pointers stay valid
        # one zeroed fp32 buffer for all tables' gradients: each block's attention backward accumulates its dRPB
        # into its slice (WindowAttnFn reads t._dfk_gview) — one fill per step instead of one per block, and the
        # backward below finds the gradients already contiguous (no cat)
        ctx.gbuf = torch.zeros_like(out)
        tabs = tuple(out[o:o + L * h].view(L, h) for o, L, h in dims)
        for t, (o, L, h) in zip(tabs, dims):
            t._dfk_gview = ctx.gbuf[o:o + L * h].view(L, h)
        return tabs

    @staticmethod
    def backward(ctx, *douts):
        saved = ctx.saved_tensors
        n = ctx.n
        out, params = saved[0], saved[1 + n + 3 * n:]
        base = ctx.gbuf.data_ptr() if ctx.gbuf is not None else -1
        if base >= 0 and all(d is not None and d.dtype == torch.float32 and d.data_ptr() == base + 4 * o
               for d, (o, L, h) in zip(douts, ctx.dims)):
            dflat = ctx.gbuf   # every block accumulated into its slice of the shared buffer
        else:
            dflat = torch.cat([(d if d is not None else torch.zeros(L, h, device=out.device)).float().reshape(-1)
                               for d, (o, L, h) in zip(douts, ctx.dims)])
        ctx.gbuf = None
        sinks = [grad_sink(p) for p in params]
        rows = [r[:4] + [t.data_ptr() for t in sinks[3 * i:3 * i + 3]] + r[7:] for i, r in enumerate(ctx.fwd_rows)]
        K.L.check(K.L.lib().dfk_cpb_bias_bwd_many(K.L.ptr(_cpb_desc(rows, out.device)), n, ctx.maxL, K.L.ptr(out),
                                                   K.L.ptr(dflat), K.L.stream()), "cpb_bias_bwd_many")
        return (None,) + (None,) * n + tuple(grad_done(p, g) for p, g in zip(params, sinks))


def cpb_tables(attns):
    """The bias tables of a list of SwinV2 WindowAttention modules in one launch each way (CPBManyFn)."""
    coords = [a.relative_coords_table for a in attns]
    params = []
    for a in attns:
        params += [a.cpb_mlp[0].weight, a.cpb_mlp[0].bias, a.cpb_mlp[2].weight]
    return CPBManyFn.apply(len(attns), *coords, *params)


class PatchEmbedLNFn(torch.autograd.Function):
    """Fused PatchEmbed3D pad + Conv3d(2x4x4) + LayerNorm in bf16 (video_swin_transformer.py:446-458):
    dfk_patch_embed_fwd reads the fp32 clip once and writes the normalised bf16 tokens once; the backward
    recomputes the conv from the clip (nothing but the LN statistics is saved) and returns the four
    parameter gradients.  -> token-major [B*Do*Ho*Wo, C] bf16."""

    @staticmethod
    def forward(ctx, x, weight, bias, ln_w, ln_b, layout, eps):
        dt = torch.bfloat16
        W = compute_weight(weight, dt).reshape(weight.shape[0], -1)
        Bc, G, Bt = (compute_weight(t, dt) for t in (bias, ln_w, ln_b))
        y, mean, rstd, grid = K.patch_embed_fwd(x, layout, W, Bc, G, Bt, eps)
        for i, p in enumerate((weight, bias, ln_w, ln_b)):
            grad_use(ctx, 1 + i, p)
        ctx.save_for_backward(x, weight, bias, ln_w, ln_b, mean, rstd)
        ctx.layout, ctx.eps = layout, eps
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, ln_w, ln_b, mean, rstd = ctx.saved_tensors
        dt = torch.bfloat16
        W = compute_weight(weight, dt).reshape(weight.shape[0], -1)
        Bc, G, Bt = (compute_weight(t, dt) for t in (bias, ln_w, ln_b))
        dw, db, dg, dbt = grad_sink(weight), grad_sink(bias), grad_sink(ln_w), grad_sink(ln_b)
        K.patch_embed_bwd(x, ctx.layout, W, Bc, G, Bt, ctx.eps, mean, rstd, dy.contiguous(), dw.view(dw.shape[0], -1),
                          db, dg, dbt)
        return (None, grad_done(weight, dw), grad_done(bias, db), grad_done(ln_w, dg), grad_done(ln_b, dbt), None,
                None)


class PatchEmbedFn(torch.autograd.Function):
    """Conv with kernel == stride as im2col + GEMM (+bias): PatchEmbed3D.proj
    (video_swin_transformer.py:436,453) / SwinV2 PatchEmbed.proj.  Returns
    token-major [B*Do*Ho*Wo, Cout].  No input gradient (the input is data)."""

    @staticmethod
    def forward(ctx, x, weight, bias, layout, patch, dtype):
        cols, grid = K.patch_im2col(x, layout, patch, dtype)
        W = compute_weight(weight, dtype).reshape(weight.shape[0], -1)
        y = K.linear(cols, W, compute_weight(bias, dtype))
        grad_use(ctx, 1, weight)
        grad_use(ctx, 2, bias)
        ctx.save_for_backward(cols, weight, bias)
        ctx.grid = grid
        return y

    @staticmethod
    def backward(ctx, dy):
        cols, weight, bias = ctx.saved_tensors
        dy = dy.contiguous()
        dw, db = grad_sink(weight), grad_sink(bias)
        K.linear_dw(dy, cols, dw.view(weight.shape[0], -1), db=db)
        return None, grad_done(weight, dw), grad_done(bias, db), None, None, None


# ---------------------------------------------------------------- 2-D convolution family
def _conv_weight2d(weight, dt):
    """[Cout, Cin, kh, kw] -> the GEMM operand [Cout, kh*kw*Cin] (tap-major, channel-fastest: im2col's columns)."""
    w = compute_weight(weight, dt)
    if w.shape[2] == 1 and w.shape[3] == 1:
        return w.reshape(w.shape[0], w.shape[1])
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


class ConvBNReLUFn(torch.autograd.Function):
    """The reference's Conv2d block (InceptionResV2.py:6-16): nn.Conv2d(bias=False) -> BatchNorm2d(eps 1e-3,
    momentum 0.1) -> ReLU on channels-last [N, H, W, C] activations.  k x k / strided convs run as im2col +
    MFMA GEMM, 1x1 stride-1 convs as the GEMM on the activation rows; training-mode BN uses batch statistics and
    updates the running ones (eval mode: the running ones)."""

    @staticmethod
    def forward(ctx, x, weight, gamma, beta, bn, k, s, p, training):
        N, H, W, C = x.shape
        dt = x.dtype
        g = K.conv2d_geo(N, H, W, C, k, s, p)
        w2 = _conv_weight2d(weight, dt)
        Cout = w2.shape[0]
        one = g.kh == 1 and g.kw == 1 and g.sh == 1 and g.sw == 1 and g.ph == 0 and g.pw == 0
        cols = x.reshape(N * H * W, C) if one and x.is_contiguous() else K.im2col2d(x, g)
        z = K.linear(cols, w2)
        y = torch.empty_like(z)
        gm, bt = gamma.detach().float(), beta.detach().float()
        if training:
            mean, rstd = K.bn2d_fwd(z, y, gm, bt, bn.eps, bn.momentum, True, bn.running_mean, bn.running_var)
        else:
            mean = bn.running_mean.float()
            rstd = torch.rsqrt(bn.running_var.float() + bn.eps)
            K.bn2d_apply(z, y, mean, rstd, gm, bt, True)
        for i, q in ((1, weight), (2, gamma), (3, beta)):
            grad_use(ctx, i, q)
        ctx.save_for_backward(cols, w2, z, y, mean, rstd, weight, gamma, beta)
        ctx.g, ctx.one, ctx.xshape = g, one, x.shape
        return y.view(N, g.Ho, g.Wo, Cout)

    @staticmethod
    def backward(ctx, dy):
        cols, w2, z, y, mean, rstd, weight, gamma, beta = ctx.saved_tensors
        g = ctx.g
        dy2 = dy.reshape(z.shape).contiguous()
        dz = torch.empty_like(z)
        dg, db = grad_sink(gamma), grad_sink(beta)
        K.bn2d_bwd(dy2, y, z, dz, mean, rstd, gamma.detach().float(), True, dg, db)
        dw = grad_sink(weight)
        kh, kw = g.kh, g.kw
        if kh == 1 and kw == 1:
            K.linear_dw(dz, cols, dw.view(dw.shape[0], -1))
        else:
            dw2 = torch.zeros(w2.shape, device=dz.device, dtype=torch.float32)
            K.linear_dw(dz, cols, dw2)
            dw += dw2.view(dw.shape[0], kh, kw, -1).permute(0, 3, 1, 2)
        dx = None
        if ctx.needs_input_grad[0]:
            dcols = K.linear_dx(dz, w2)
            if ctx.one:
                dx = dcols.view(ctx.xshape)
            else:
                dx = torch.empty(ctx.xshape, device=dz.device, dtype=dz.dtype)
                K.col2im2d(dcols, g, dx)
        return dx, grad_done(weight, dw), grad_done(gamma, dg), grad_done(beta, db), None, None, None, None, None


class ResConvFn(torch.autograd.Function):
    """Inception-ResNet residual (InceptionResV2.py:90-95,112-117,159-166): y = relu?(x + scale * conv1x1(x_res)),
    the conv with bias, as one GEMM with the scale / residual / ReLU epilogue."""

    @staticmethod
    def forward(ctx, xres, weight, bias, x, scale, relu):
        N, H, W, C = x.shape
        dt = x.dtype
        w2 = _conv_weight2d(weight, dt)
        a = xres.reshape(-1, xres.shape[-1])
        y = torch.empty(N * H * W, C, device=x.device, dtype=dt)
        K.gemm(a, a.stride(0), False, w2, w2.stride(0), False, a.shape[0], C, a.shape[1], y, C, dtype=K.L.dt(x),
               bias=compute_weight(bias, dt), residual=x.reshape(-1, C), ldr=C, act=3 if relu else 0,
               alpha=float(scale))
        for i, q in ((1, weight), (2, bias)):
            grad_use(ctx, i, q)
        ctx.save_for_backward(a, w2, y, weight, bias)
        ctx.scale, ctx.relu, ctx.xres_shape = float(scale), relu, xres.shape
        return y.view(N, H, W, C)

    @staticmethod
    def backward(ctx, dy):
        a, w2, y, weight, bias = ctx.saved_tensors
        dy2 = dy.reshape(y.shape)
        if ctx.relu:
            dy2 = dy2 * (y > 0).to(dy2.dtype)
        dy2 = dy2.contiguous()
        dz = (dy2 * ctx.scale).contiguous()
        dw, db = grad_sink(weight), grad_sink(bias)
        K.linear_dw(dz, a, dw.view(dw.shape[0], -1), db=db)
        dxres = K.linear_dx(dz, w2).view(ctx.xres_shape)
        return dxres, grad_done(weight, dw), grad_done(bias, db), dy2.view(dy.shape), None, None


class Pool2dFn(torch.autograd.Function):
    """MaxPool2d(3, s, 0) (mode 0) / AvgPool2d(3, 1, 1, count_include_pad=False) (mode 1) on [N, H, W, C]."""

    @staticmethod
    def forward(ctx, x, k, s, p, mode):
        N, H, W, C = x.shape
        g = K.conv2d_geo(N, H, W, C, k, s, p)
        ctx.save_for_backward(x)
        ctx.g, ctx.mode = g, mode
        return K.pool2d_fwd(x, g, mode)

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        return K.pool2d_bwd(x, dy.contiguous(), ctx.g, ctx.mode), None, None, None, None
