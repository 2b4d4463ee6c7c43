"""Thin tensor-level wrappers over the C ABI (include/dfk.h).

Every function enqueues on torch's current HIP stream, allocates outputs with
the torch caching allocator (graph-capture safe) and raises on any error.
Activations are 2-D token-major views ([rows, C], contiguous rows).
"""
import ctypes
import math
import os

import torch

from . import _lib as L

# split-K target grid of a skinny weight-gradient GEMM: 256 workgroups.  In isolation 512 (two per CU) runs each
# dW fastest, but inside the step the other two branch streams fill the chip and fewer splits mean fewer fp32
# partials (whole-step A/B, C2: 512 / 256 / 128 = 241.7 / 244.8 / 245.3 clips/s, 64: 232.7; C4 Swin-B:
# 134.1 / 133.1 / 124.3 — 256 holds both; round 4, r4tg: C2 160 / 256 = 257.9 / 256.7, C4 134.1 / 139.2)
_CU_TARGET_BLOCKS = int(os.environ.get("DFK_DW_TARGET", "256"))


def _view(t, ld, bs0=0, bs1=0, conv=None):
    v = L.View()
    v.ptr = t.data_ptr()
    v.ld, v.bs0, v.bs1 = int(ld), int(bs0), int(bs1)
    if conv:
        v.conv_cg, v.conv_stride, v.conv_pad, v.conv_rows = (int(c) for c in conv)
    return v


def gemm(a, a_ld, a_kmajor, b, b_ld, b_kmajor, M, N, K, c, ldc, *, dtype, c_f32=False, bias=None,
         residual=None, ldr=0, aux=None, ldaux=0, act=0, beta=0.0, atomic=False, splitk=1,
         nz=(1, 1), a_bs=(0, 0), b_bs=(0, 0), c_bs=(0, 0), r_bs=(0, 0), a_conv=None, b_conv=None, bias_bs1=0,
         rowsum=None, drop=None, alpha=0.0):
    """Raw dfk_gemm.  a/b/c are tensors (base pointers); see include/dfk.h.  drop: rng.Drop spec of the
    output's dropout / DropPath (applied before the residual add)."""
    g = L.GemmArgs()
    if drop is not None:
        g.drop = L.drop(drop, c.device)
    g.bias_bs1 = int(bias_bs1)
    g.a = _view(a, a_ld, *a_bs, conv=a_conv)
    g.b = _view(b, b_ld, *b_bs, conv=b_conv)
    g.c = c.data_ptr()
    g.bias = bias.data_ptr() if bias is not None else None
    g.residual = residual.data_ptr() if residual is not None else None
    g.aux = aux.data_ptr() if aux is not None else None
    g.ldc, g.cbs0, g.cbs1 = int(ldc), int(c_bs[0]), int(c_bs[1])
    g.ldr, g.rbs0, g.rbs1 = int(ldr), int(r_bs[0]), int(r_bs[1])
    g.ldaux = int(ldaux)
    g.M, g.N, g.K = int(M), int(N), int(K)
    g.dtype = dtype
    g.a_kmajor, g.b_kmajor = int(a_kmajor), int(b_kmajor)
    g.c_f32 = int(c_f32)
    g.nz0, g.nz1 = int(nz[0]), int(nz[1])
    g.splitk = int(splitk)
    g.act = int(act)
    g.atomic = int(atomic)
    g.beta = float(beta)
    g.rowsum = rowsum.data_ptr() if rowsum is not None else None
    g.alpha = float(alpha)
    for t in (a, b, c):
        if not t.is_cuda:
            raise RuntimeError("deepfake_amd: tensors must be on the HIP device (no CPU fallback)")
    ws = None
    nbytes = L.lib().dfk_gemm_workspace(g)
    if nbytes > 0:
        ws = torch.empty(nbytes // 4, device=c.device, dtype=torch.float32)
        g.ws = ws.data_ptr()
    L.check(L.lib().dfk_gemm(g, L.stream()), f"gemm M={M} N={N} K={K}")


def linear(x, w, b=None, act=0, aux=None, residual=None, out=None, beta=0.0, drop=None):
    """y[M,N] = x[M,K] @ w[N,K]^T (+b) (gelu: act=1, preact -> aux) (dropout) (+residual)."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    gemm(x, x.stride(0), False, w, w.stride(0), False, M, N, K, out, out.stride(0), dtype=L.dt(x), bias=b,
         residual=residual, ldr=residual.stride(0) if residual is not None else 0, aux=aux,
         ldaux=aux.stride(0) if aux is not None else 0, act=act, beta=beta, drop=drop)
    return out


class MxTensor:
    """An MX-fp8 operand (include/dfk.h dfk_mx_operand): e4m3 values q [rows, K] (uint8, K contiguous) and the
    E8M0 block scales s [K/128, rows] (int32: four bytes = the four 32-blocks of one 128-k tile)."""

    def __init__(self, q, s):
        self.q, self.s = q, s

    @property
    def shape(self):
        return tuple(self.q.shape)

    def operand(self):
        o = L.MxOperand()
        o.q, o.s = self.q.data_ptr(), self.s.data_ptr()
        o.ld, o.lds = int(self.q.stride(0)), int(self.s.stride(0))
        return o


def mx_quant(x, transpose=False):
    """x [rows, cols] (bf16 / fp32, unit stride along cols) -> MxTensor along cols ([rows, cols]), or along rows
    of x^T (transpose=True: [cols, rows]; the dX GEMM's W^T)."""
    rows, cols = x.shape
    if x.stride(1) != 1:
        x = x.contiguous()
    R, Kd = (cols, rows) if transpose else (rows, cols)
    if Kd % 128:
        raise ValueError(f"mx_quant: the quantised dim ({Kd}) must be a multiple of 128")
    q = torch.empty(R, Kd, device=x.device, dtype=torch.uint8)
    s = torch.empty(Kd // 128, R, device=x.device, dtype=torch.int32)
    L.check(L.lib().dfk_mx_quant(L.ptr(x), L.dt(x), rows, cols, x.stride(0), int(transpose), L.ptr(q), q.stride(0),
                                 L.ptr(s), L.stream()), "mx_quant")
    return MxTensor(q, s)


def mx_empty(rows, K, device):
    return MxTensor(torch.empty(rows, K, device=device, dtype=torch.uint8),
                    torch.empty(K // 128, rows, device=device, dtype=torch.int32))


def gemm_mx(a, b, out=None, bias=None, act=0, aux=None, residual=None, drop=None, beta=0.0, mx_out=False):
    """out [M, N] bf16 = A B^T (+ the dfk_gemm epilogue) with A [M, K], B [N, K] MxTensors (dfk_gemm_mx).
    mx_out=True: also return the output quantised along N (the next MX GEMM's A operand), from the same
    epilogue: (out, MxTensor)."""
    M, Kd = a.shape
    N = b.shape[0]
    if b.shape[1] != Kd:
        raise ValueError(f"gemm_mx: K mismatch {a.shape} x {b.shape}")
    if out is None:
        out = torch.empty(M, N, device=a.q.device, dtype=torch.bfloat16)
    g = L.GemmArgs()
    if drop is not None:
        g.drop = L.drop(drop, out.device)
    g.c = out.data_ptr()
    g.bias = bias.data_ptr() if bias is not None else None
    g.residual = residual.data_ptr() if residual is not None else None
    g.aux = aux.data_ptr() if aux is not None else None
    g.ldc = int(out.stride(0))
    g.ldr = int(residual.stride(0)) if residual is not None else 0
    g.ldaux = int(aux.stride(0)) if aux is not None else 0
    g.M, g.N, g.K = int(M), int(N), int(Kd)
    g.dtype = L.BF16
    g.nz0 = g.nz1 = 1
    g.splitk = 1
    g.act = int(act)
    g.beta = float(beta)
    for t in (bias, residual, aux):
        if t is not None and t.dtype != torch.bfloat16:
            raise TypeError("gemm_mx: the epilogue operands are bf16")
    mo = None
    if mx_out:
        if N % 128:
            raise ValueError(f"gemm_mx: an MX copy of the output needs N % 128 == 0 (N={N})")
        mo = mx_empty(M, N, out.device)
        g.mx_q, g.mx_s = mo.q.data_ptr(), mo.s.data_ptr()
        g.mx_ldq, g.mx_lds = int(mo.q.stride(0)), int(mo.s.stride(0))
    L.check(L.lib().dfk_gemm_mx(g, a.operand(), b.operand(), L.stream()), f"gemm_mx M={M} N={N} K={Kd}")
    return (out, mo) if mx_out else out


def linear_dx(dy, w, out=None, act=0, aux=None, beta=0.0, drop=None, residual=None):
    """dx[M,K] = dy[M,N] @ w[N,K]  (act=2: times gelu'(aux)) (drop: times the forward's dropout mask)
    (+ residual[M,K]: the gradient the input receives along a skip path, added in the epilogue)."""
    M, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=dy.dtype)
    if residual is not None:
        residual = residual.contiguous()
    if (_DX_BLAS and act == 0 and beta == 0.0 and drop is None and residual is None and M <= _DX_BLAS_MAX_M
            and dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and dy.is_contiguous() and out.is_contiguous()):
        # a plain product with no epilogue on the small-M shapes: the vendor library (hipBLASLt) runs it faster
        # than the LDS-DMA kernel there (profiles/gemm/r6z_gemm_vs_hipblaslt.txt); the fused forms stay on dfk_gemm
        return torch.matmul(dy, w, out=out)
    gemm(dy, dy.stride(0), False, w, w.stride(0), True, M, K, N, out, out.stride(0), dtype=L.dt(dy), act=act,
         aux=aux, ldaux=aux.stride(0) if aux is not None else 0, beta=beta, drop=drop, residual=residual,
         ldr=residual.stride(0) if residual is not None else 0)
    return out


_DX_BLAS = os.environ.get("DFK_DX_BLAS", "1") == "1"   # plain small-M dX products on hipBLASLt (DFK_DX_BLAS=0: dfk_gemm)
_DX_BLAS_MAX_M = int(os.environ.get("DFK_DX_BLAS_MAX_M", "131072"))
_DW_MIN_K = int(os.environ.get("DFK_DW_MINK", "512"))   # tokens per split of a weight-gradient GEMM (tuning)
_DW_UNSPLIT64 = int(os.environ.get("DFK_DW_UNSPLIT64", "384"))   # 64x64 tiles from which dW runs unsplit (r5o: the
# 256-tile SwinV2 stage-3 fc1 / fc2 dW 22 -> 19, 21 -> 19 us on split 128x128 tiles; w2v (432-576 tiles) flat)
_DW_XCD = int(os.environ.get("DFK_DW_XCD", "1"))   # split counts rounded to multiples of 8 (XCD grouping; A/B knob)
_DW_SLAB = os.environ.get("DFK_DW_SLAB", "0") == "1"   # fp32 split slabs + one reduce instead of split atomics (A/B knob)


def splitk_for(tiles, K, min_k=None):
    min_k = _DW_MIN_K if min_k is None else min_k
    return max(1, min(_CU_TARGET_BLOCKS // max(tiles, 1), max(K // min_k, 1)))


def linear_dw(dy, x, dw, db=None):
    """dw[N,K] (fp32, +=) += dy[M,N]^T @ x[M,K]; with db [N] fp32: db += column sums of dy (the bias
    gradient) from the same pass over dy.  Output grids that fill the chip run unsplit and add in the
    epilogue; skinny ones split the M reduction and add fp32 partials atomically."""
    M, N = dy.shape
    K = x.shape[1]
    if math.ceil(N / 64) * math.ceil(K / 64) >= _DW_UNSPLIT64:
        gemm(dy, dy.stride(0), True, x, x.stride(0), True, N, K, M, dw, dw.stride(0), dtype=L.dt(dy), c_f32=True,
             beta=1.0, rowsum=db)
        return dw
    tiles = math.ceil(N / 128) * math.ceil(K / 128)
    s = splitk_for(tiles, M)
    # fp32 partial bytes (splits x N x K x 4) kept to a quarter of the operand bytes read, except that small
    # grids keep up to 8 splits for parallelism (C2 sweep: mel1.fc1 [25088]x512x128 98 -> 30 splits, 42 -> 28 us)
    s = max(1, min(s, max(8, M * (N + K) // (8 * N * K))))
    if _DW_XCD and tiles > 1 and s >= 16:
        s -= s % 8   # a multiple of 8 splits: the kernel puts each split's tiles on one XCD (shared operand in L2)
    slab = s > 1 and _DW_SLAB   # A/B: fp32 split slabs + one reduce pass instead of the splits' fp32 atomics
    gemm(dy, dy.stride(0), True, x, x.stride(0), True, N, K, M, dw, dw.stride(0), dtype=L.dt(dy), c_f32=True,
         atomic=s > 1 and not slab, beta=1.0, splitk=s, rowsum=db)
    return dw


def colsum(x, out):
    """out[j] (fp32) += sum_i x[i, j]."""
    rows, cols = x.shape
    L.check(L.lib().dfk_colsum(L.ptr(x), L.dt(x), rows, cols, x.stride(0), L.ptr(out), L.stream()), "colsum")
    return out


def layernorm_fwd(x, w, b, eps=1e-5, out=None, residual=None, drop=None):
    """y = LN(x) (residual + drop(LN(x)) with residual / drop)."""
    rows, C = x.shape
    if out is None:
        out = torch.empty_like(x)
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    d = L.drop(drop, x.device)
    L.check(L.lib().dfk_layernorm_fwd(L.ptr(x), L.ptr(w), L.ptr(b), L.ptr(out), L.ptr(mean), L.ptr(rstd), rows, C,
                                      float(eps), L.dt(x), L.ptr(residual), d, L.stream()), "layernorm_fwd")
    return out, mean, rstd


# LayerNorms of <= 4096 rows: at most _LN_SMALL workgroups with atomic dw/db partials (layernorm.hip bwd_blocks)
_LN_SMALL = int(os.environ.get("DFK_LN_SMALL", "128"))
_LN_SMALL_ROWS = 4096


def _ln_bwd_blocks(rows, C):
    """Workgroups of ln_bwd (layernorm.hip bwd_blocks)."""
    nv = C // 8
    lanes = 16 if nv <= 16 else (32 if nv <= 32 else 64)
    return min(2048, -(-rows // (4 * (64 // lanes))))


def layernorm_bwd(dy, x, w, mean, rstd, dw, db, dx=None, accumulate=False, slab_partials=None, drop=None,
                  addend=None):
    """dx (+)= LN backward (+ addend [rows, C] of x's dtype, read: the skip path's gradient summed in the same
    pass without writing into it); dw / db (fp32) += the affine gradients.  slab_partials (default: from 64
    workgroups up) writes each workgroup's dw/db partial to a slab summed by a column pass instead of adding
    it atomically: hundreds of workgroups adding into the same C addresses serialise on a few L2 channels
    (the 1568 x 512 SwinV2 / wav2vec2 LNs ran 20 us, the 401k x 96 stage-1 LN 116 us)."""
    rows, C = x.shape
    if dx is None:
        dx = torch.empty_like(x)
    if slab_partials is None:
        slab_partials = _ln_bwd_blocks(rows, C) >= 64 and not (_LN_SMALL > 0 and rows <= _LN_SMALL_ROWS)
    ws = None
    if slab_partials and (dw is not None or db is not None):   # per-workgroup dw/db partials + column sums
        ws = torch.empty(max(L.lib().dfk_layernorm_bwd_workspace(rows, C) // 4, 1), device=x.device,
                         dtype=torch.float32)
    L.check(L.lib().dfk_layernorm_bwd(L.ptr(dy), L.ptr(x), L.ptr(w), L.ptr(mean), L.ptr(rstd), L.ptr(dx),
                                      L.ptr(dw), L.ptr(db), rows, C, int(accumulate), L.dt(x), L.ptr(ws),
                                      L.drop(drop, x.device), L.ptr(addend), L.stream()), "layernorm_bwd")
    return dx


def wattn_args(q, k, v, out, ld_qkv, dims, window, full_window, shift, heads, hd, scale, rpb=None, pads=None,
               lse=None, mask=None, drop=None):
    a = L.WattnArgs()
    if drop is not None:
        a.drop = L.drop(drop, q.device)
    if mask is not None:
        a.mask, a.mask_nw = mask.data_ptr(), int(mask.shape[0])
    a.q, a.k, a.v, a.out = q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr()
    a.rpb = rpb.data_ptr() if rpb is not None else None
    if pads is not None:
        a.pad_q, a.pad_k, a.pad_v = (p.data_ptr() for p in pads)
    a.lse = lse.data_ptr() if lse is not None else None
    a.ld_qkv, a.ld_out = int(ld_qkv), int(out.stride(-2) if out.dim() > 1 else heads * hd)
    a.B, a.D, a.H, a.W = (int(d) for d in dims)
    a.wd, a.wh, a.ww = (int(w) for w in window)
    a.fd, a.fh, a.fw = (int(w) for w in full_window)
    a.sd, a.sh, a.sw = (int(s) for s in shift)
    a.heads, a.hd = int(heads), int(hd)
    a.dtype = L.dt(q)
    a.scale = float(scale)
    return a


def window_geometry(dims, window):
    B, D, H, W = dims
    Dp, Hp, Wp = (math.ceil(n / w) * w for n, w in zip((D, H, W), window))
    nW = (Dp // window[0]) * (Hp // window[1]) * (Wp // window[2])
    N = window[0] * window[1] * window[2]
    Np = math.ceil(N / 32) * 32
    return nW, N, Np


def wattn_fwd(q, k, v, ld_qkv, dims, window, full_window, shift, heads, hd, scale, rpb=None, pads=None,
              out=None, need_lse=True, mask=None, use_table=True, return_table=False, tab=None, drop=None):
    """Token-major window attention core; returns (out [rows, heads*hd], lse[, tab]).
    use_table: bf16 score-bias tables (RPB + shift mask per shift class, built by dfk_wattn_table, or
    `tab` from an earlier call with the same geometry and rpb); the backward must get the same `tab`."""
    rows = dims[0] * dims[1] * dims[2] * dims[3]
    if out is None:
        out = torch.empty(rows, heads * hd, device=q.device, dtype=q.dtype)
    nW, N, Np = window_geometry(dims, window)
    lse = torch.empty(dims[0] * nW * heads, Np, device=q.device, dtype=torch.float32) if need_lse else None
    a = wattn_args(q, k, v, out, ld_qkv, dims, window, full_window, shift, heads, hd, scale, rpb, pads, lse, mask,
                   drop)
    if tab is not None:
        a.tab = tab.data_ptr()
    elif use_table and os.environ.get("DFK_WATTN_TABLE", "1") != "0":
        nbytes = L.lib().dfk_wattn_table_workspace(a)
        if nbytes < 0:
            raise RuntimeError("dfk_wattn_table_workspace: invalid arguments")
        if nbytes > 0:
            tab = torch.empty(nbytes // 4, device=q.device, dtype=torch.float32)
            a.tab = tab.data_ptr()
            L.check(L.lib().dfk_wattn_table(a, L.stream()), "wattn_table")
    L.check(L.lib().dfk_wattn_fwd(a, L.stream()), "wattn_fwd")
    if return_table:
        return out, lse, tab
    return out, lse


def wattn_fwd_policy(version=-1, bal_min_units=-1):
    """Process-wide kernel choice of the hd-32 bf16 table forward (tests / A/B runs): version 6 (no running max,
    16x16x32 tiles, default), 5 (32x32x16) or 4 (max-subtracted); bal_min_units = smallest launch on the balanced
    key-split schedule. -1 leaves a setting, -2 restores the default.  The bias table must be built under the same policy as the forward."""
    L.check(L.lib().dfk_wattn_fwd_policy(int(version), int(bal_min_units)), "wattn_fwd_policy")


def wattn_bwd_policy(group=0, version=-1):
    """Process-wide backward policy (tests / A/B runs): windows per workgroup whose dS^T share one dRPB scratch
    slab (0 restores the automatic choice); version 4 (two-pass kernel, default) or 3 (staggered single pass),
    -1 leaves it."""
    L.check(L.lib().dfk_wattn_bwd_policy(int(group), int(version)), "wattn_bwd_policy")


def wattn_bwd(fwd_args_tensors, dout, dq, dk, dv, ld_dqkv, drpb=None, dpads=None, mask=None, tab=None, drop=None,
              dscore=None):
    """Backward of wattn_fwd.  fwd_args_tensors = (q, k, v, out, lse, ld_qkv, dims, window, full_window,
    shift, heads, hd, scale, rpb, pads).  dq/dk/dv may alias column slices of one [rows, 3C] buffer."""
    (q, k, v, out, lse, ld_qkv, dims, window, full_window, shift, heads, hd, scale, rpb, pads) = fwd_args_tensors
    ba = L.WattnBwdArgs()
    ba.f = wattn_args(q, k, v, out, ld_qkv, dims, window, full_window, shift, heads, hd, scale, rpb, pads, lse, mask,
                      drop)
    if tab is not None:
        ba.f.tab = tab.data_ptr()
    ba.dout = dout.data_ptr()
    ba.dq, ba.dk, ba.dv = dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
    ba.drpb = drpb.data_ptr() if drpb is not None else None
    if dpads is not None:
        ba.dpad_q, ba.dpad_k, ba.dpad_v = (p.data_ptr() for p in dpads)
    ba.ld_dqkv = int(ld_dqkv)
    ba.ld_dout = int(dout.stride(0))
    ba.dscore = dscore.data_ptr() if dscore is not None else None
    ws = None
    if drpb is not None:
        nbytes = L.lib().dfk_wattn_bwd_workspace(ba.f)
        if nbytes < 0:
            raise RuntimeError("dfk_wattn_bwd_workspace: invalid arguments")
        ws = torch.empty(max(nbytes // 4, 1), device=dout.device, dtype=torch.float32)
        ba.ws = ws.data_ptr()
    L.check(L.lib().dfk_wattn_bwd(ba, L.stream()), "wattn_bwd")


def patch_im2col(x, layout, patch, out_dtype):
    """x: video [B,T,C,H,W] (layout 'btchw') or [B,C,T,H,W] ('bcthw') or image [B,C,H,W] ('bchw').
    Returns (cols [B*Do*Ho*Wo, C*pd*ph*pw], (B, Do, Ho, Wo))."""
    a = L.Im2colArgs()
    if layout == "bchw":
        B, Cin, H, W = x.shape
        T = 1
        sb, sc, sh, sw = x.stride()
        st = 0
        pd, ph, pw = 1, patch[0], patch[1]
    else:
        if layout == "btchw":
            B, T, Cin, H, W = x.shape
            sb, st, sc, sh, sw = x.stride()
        else:
            B, Cin, T, H, W = x.shape
            sb, sc, st, sh, sw = x.stride()
        pd, ph, pw = patch
    Do, Ho, Wo = -(-T // pd), -(-H // ph), -(-W // pw)
    a.sb, a.sc, a.st, a.sh, a.sw = sb, sc, st, sh, sw
    a.B, a.cin, a.T, a.H, a.W = B, Cin, T, H, W
    a.pd, a.ph, a.pw = pd, ph, pw
    a.Do, a.Ho, a.Wo = Do, Ho, Wo
    out = torch.empty(B * Do * Ho * Wo, Cin * pd * ph * pw, device=x.device, dtype=out_dtype)
    L.check(L.lib().dfk_patch_im2col(L.ptr(x), L.dt(x), L.ptr(out), L.dt(out), a, L.stream()), "patch_im2col")
    return out, (B, Do, Ho, Wo)


def patch_embed_args(x, layout, w, b, ln_w, ln_b, eps):
    """dfk_patch_embed_args for a [B,T,3,H,W] ('btchw') or [B,3,T,H,W] ('bcthw') fp32 clip."""
    a = L.PatchEmbedArgs()
    if layout == "btchw":
        B, T, _, H, W = x.shape
        a.sb, a.st, a.sc, a.sh, a.sw = x.stride()
    else:
        B, _, T, H, W = x.shape
        a.sb, a.sc, a.st, a.sh, a.sw = x.stride()
    a.x = x.data_ptr()
    a.B, a.T, a.H, a.W, a.C = B, T, H, W, w.shape[0]
    a.w, a.b, a.ln_w, a.ln_b = w.data_ptr(), b.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr()
    a.eps = float(eps)
    return a, (B, -(-T // 2), -(-H // 4), -(-W // 4))


def patch_embed_fwd(x, layout, w, b, ln_w, ln_b, eps):
    """Fused pad + Conv3d(2x4x4) + LayerNorm -> (tokens [B*Do*Ho*Wo, C] bf16, mean, rstd, grid)."""
    a, grid = patch_embed_args(x, layout, w, b, ln_w, ln_b, eps)
    rows = grid[0] * grid[1] * grid[2] * grid[3]
    out = torch.empty(rows, w.shape[0], device=x.device, dtype=torch.bfloat16)
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    a.out, a.mean, a.rstd = out.data_ptr(), mean.data_ptr(), rstd.data_ptr()
    L.check(L.lib().dfk_patch_embed_fwd(a, L.stream()), "patch_embed_fwd")
    return out, mean, rstd, grid


def patch_embed_bwd(x, layout, w, b, ln_w, ln_b, eps, mean, rstd, dy, dw, db, dln_w, dln_b):
    a, _ = patch_embed_args(x, layout, w, b, ln_w, ln_b, eps)
    a.mean, a.rstd = mean.data_ptr(), rstd.data_ptr()
    a.dw, a.db, a.dln_w, a.dln_b = dw.data_ptr(), db.data_ptr(), dln_w.data_ptr(), dln_b.data_ptr()
    L.check(L.lib().dfk_patch_embed_bwd(a, L.ptr(dy), L.stream()), "patch_embed_bwd")


def patch_merge(x, dims, reverse=False, out=None):
    """dims = (B, D, H, W) of the un-merged volume; x token-major rows (or merged rows when reverse)."""
    B, D, H, W = dims
    C = x.shape[1] if not reverse else x.shape[1] // 4
    if out is None:
        if reverse:   # every un-merged token belongs to exactly one merged row: the kernel writes all of out
            out = torch.empty(B * D * H * W, C, device=x.device, dtype=x.dtype)
        else:
            out = torch.empty(B * D * ((H + 1) // 2) * ((W + 1) // 2), 4 * C, device=x.device, dtype=x.dtype)
    L.check(L.lib().dfk_patch_merge(L.ptr(x), L.ptr(out), B, D, H, W, C, int(reverse), L.dt(x), L.stream()),
            "patch_merge")
    return out


def rowmean(x, groups, out_f32=True):
    rows, C = x.shape
    R = rows // groups
    out = torch.empty(groups, C, device=x.device, dtype=torch.float32 if out_f32 else x.dtype)
    L.check(L.lib().dfk_rowmean(L.ptr(x), L.ptr(out), groups, R, C, L.dt(x), int(out.dtype == torch.float32),
                                L.stream()), "rowmean")
    return out


def w2v_conv0_fwd(wave, w, gamma, beta, eps, dtype):
    B, S = wave.shape
    T0 = (S - 10) // 5 + 1
    out = torch.empty(B, T0, 512, device=wave.device, dtype=dtype)
    stats = torch.empty(B, 512, 2, device=wave.device, dtype=torch.float32)
    ws = torch.empty(max(L.lib().dfk_w2v_conv0_fwd_workspace(B, S) // 4, 1), device=wave.device, dtype=torch.float32)
    L.check(L.lib().dfk_w2v_conv0_fwd(L.ptr(wave), B, S, L.ptr(w), L.ptr(gamma), L.ptr(beta), float(eps),
                                      L.ptr(stats), L.ptr(out), L.dt(out), L.ptr(ws), L.stream()), "w2v_conv0_fwd")
    return out, stats


def w2v_conv0_bwd(wave, w, gamma, beta, eps, stats, dout, dw, dgamma, dbeta):
    B, S = wave.shape
    scratch = torch.empty(max(L.lib().dfk_w2v_conv0_bwd_workspace(B, S) // 4, B * 512 * 2), device=wave.device,
                          dtype=torch.float32)
    L.check(L.lib().dfk_w2v_conv0_bwd(L.ptr(wave), B, S, L.ptr(w), L.ptr(gamma), L.ptr(beta), float(eps),
                                      L.ptr(stats), L.ptr(dout), L.dt(dout), L.ptr(scratch),
                                      scratch.numel() * 4, L.ptr(dw), L.ptr(dgamma),
                                      L.ptr(dbeta), L.stream()), "w2v_conv0_bwd")


def gelu_bwd(dy, pre, out=None):
    if out is None:
        out = torch.empty_like(dy)
    L.check(L.lib().dfk_gelu_bwd(L.ptr(dy), L.ptr(pre), L.ptr(out), dy.numel(), L.dt(dy), L.stream()), "gelu_bwd")
    return out


def posconv_wnorm_fwd(v, g, C, Cg, k, norm, ws, w2, w3):
    """norm[k] = ||v[:, :, k]||; w = g v / norm into the positional conv's two GEMM operand layouts (dfk.h)."""
    L.check(L.lib().dfk_posconv_wnorm_fwd(L.ptr(v), L.ptr(g), C, Cg, k, L.ptr(norm), L.ptr(ws), L.ptr(w2), L.ptr(w3),
                                          L.dt(w2), L.stream()), "posconv_wnorm_fwd")


def posconv_wnorm_bwd(v, g, norm, dw2, C, Cg, k, ws, dv, dg):
    """dv / dg (fp32, +=) of w = g v / ||v|| from dw2 [C, k*Cg] (the dW GEMM's output in w2's layout)."""
    L.check(L.lib().dfk_posconv_wnorm_bwd(L.ptr(v), L.ptr(g), L.ptr(norm), L.ptr(dw2), C, Cg, k, L.ptr(ws), L.ptr(dv),
                                          L.ptr(dg), L.stream()), "posconv_wnorm_bwd")


def cast(x, dtype):
    y = torch.empty(x.shape, device=x.device, dtype=dtype)
    L.check(L.lib().dfk_cast(L.ptr(x), L.dt(x), L.ptr(y), L.dt(y), x.numel(), L.stream()), "cast")
    return y


def frame_normalize(frames_u8, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    """uint8 [..., H, W, 3] decoded RGB frames -> fp32 [..., 3, H, W] = (x/255 - mean) / std
    (T.ToTensor + T.Normalize, data/data_process.py:55-69)."""
    import ctypes
    *lead, H, W, c3 = frames_u8.shape
    if c3 != 3 or frames_u8.dtype != torch.uint8:
        raise ValueError("frame_normalize expects uint8 [..., H, W, 3]")
    x = frames_u8.contiguous()
    out = torch.empty(*lead, 3, H, W, device=x.device, dtype=torch.float32)
    m = (ctypes.c_float * 3)(*mean)
    s = (ctypes.c_float * 3)(*std)
    L.check(L.lib().dfk_frame_normalize(L.ptr(x), L.ptr(out), x.numel() // (3 * H * W), H, W, m, s, L.stream()),
            "frame_normalize")
    return out


def wave_normalize(wave, eps=1e-7):
    """[B, S] fp32 (zero-padded rows) -> per-row (x - mean) / sqrt(var + eps)."""
    x = wave.float().contiguous()
    out = torch.empty_like(x)
    L.check(L.lib().dfk_wave_normalize(L.ptr(x), L.ptr(out), x.shape[0], x.shape[1], float(eps), L.stream()),
            "wave_normalize")
    return out


def sgd_step(param, grad, buf, shadow, lr, momentum, wd, first, lr_dev=None, gate=None, grad_scale=1.0,
             grad_bf16=None):
    """grad_scale / grad_bf16: the data-parallel fold (gradient = grad_bf16 or grad, times grad_scale)."""
    L.check(L.lib().dfk_sgd_step(L.ptr(param), L.ptr(grad), L.ptr(buf), L.ptr(shadow) if shadow is not None else None,
                                 param.numel(), L.ptr(lr_dev) if lr_dev is not None else None, float(lr),
                                 float(momentum), float(wd), int(first), L.ptr(gate), float(grad_scale),
                                 L.ptr(grad_bf16) if grad_bf16 is not None else None, L.stream()), "sgd_step")


SGD_MAX_RUNS = 64   # dfk_sgd_step_runs' by-value run table


def sgd_step_runs(param, grad, buf, shadow, runs, momentum, wd, lr_dev, grad_scale=1.0, grad_bf16=None):
    """Every run [(start, end, gate tensor or None, first)] of one SGD step in one launch (same per-element
    arithmetic as sgd_step); the run table is host data copied into the launch arguments."""
    if not 0 < len(runs) <= SGD_MAX_RUNS:
        raise ValueError(f"sgd_step_runs takes 1..{SGD_MAX_RUNS} runs")
    tab = (ctypes.c_int64 * (4 * len(runs)))(*[v for s, e, g, f in runs
                                          for v in (s, e - s, g.data_ptr() if g is not None else 0, int(bool(f)))])
    L.check(L.lib().dfk_sgd_step_runs(L.ptr(param), L.ptr(grad), L.ptr(buf), L.ptr(shadow) if shadow is not None
                                      else None, tab, len(runs), L.ptr(lr_dev), 0.0, float(momentum), float(wd),
                                      float(grad_scale), L.ptr(grad_bf16) if grad_bf16 is not None else None,
                                      L.stream()), "sgd_step_runs")


def dropout(x, drop, out=None, group_rows=None):
    """out = x * mask / (1 - p) over a 2-D [rows, cols] view (out may be x)."""
    rows, cols = x.shape
    if out is None:
        out = torch.empty_like(x)
    L.check(L.lib().dfk_dropout(L.ptr(x), L.ptr(out), rows, cols, x.stride(0), L.drop(drop, x.device), L.dt(x),
                                L.stream()), "dropout")
    return out


def bernoulli_flags(drop, n, device):
    """fp32 [n] of 1 (keep) / 0 (drop) coins (LayerDrop)."""
    out = torch.empty(n, device=device, dtype=torch.float32)
    L.check(L.lib().dfk_bernoulli_flags(L.drop(drop, device), n, L.ptr(out), L.stream()), "bernoulli_flags")
    return out


def layer_select(y, x, keep, out=None):
    """out = y if keep[0] > 0 else x (device flag, no host sync)."""
    if out is None:
        out = torch.empty_like(y)
    L.check(L.lib().dfk_layer_select(L.ptr(y), L.ptr(x), L.ptr(keep), L.ptr(out), None, y.numel() * y.element_size(),
                                     L.stream()), "layer_select")
    return out


def layer_select_bwd(g, keep):
    """(the layer's gradient, the skip path's gradient) of layer_select."""
    gy, gx = torch.empty_like(g), torch.empty_like(g)
    L.check(L.lib().dfk_layer_select(L.ptr(g), None, L.ptr(keep), L.ptr(gy), L.ptr(gx), g.numel() * g.element_size(),
                                     L.stream()), "layer_select_bwd")
    return gy, gx


def layerdrop_flags(drop, keep, used):
    """keep[i] = coin i (1 keep / 0 drop), used[i] = max(used[i], keep[i]) — LayerDrop for one micro-step."""
    L.check(L.lib().dfk_layerdrop_flags(L.drop(drop, keep.device), keep.numel(), L.ptr(keep), L.ptr(used),
                                        L.stream()), "layerdrop_flags")


def spec_augment_fwd(h, embed, mask_prob, mask_length, min_masks, drop):
    """h [B, T, C] -> (masked copy, mask [B, T] uint8)."""
    B, T, C = h.shape
    out = torch.empty_like(h)
    mask = torch.empty(B, T, device=h.device, dtype=torch.uint8)
    L.check(L.lib().dfk_spec_augment_fwd(L.ptr(h), L.ptr(out), L.ptr(mask), L.ptr(embed), B, T, C, float(mask_prob),
                                         int(mask_length), int(min_masks), L.drop(drop, h.device), L.dt(h),
                                         L.stream()), "spec_augment_fwd")
    return out, mask


def spec_augment_bwd(dy, mask, dembed):
    B, T, C = dy.shape
    dx = torch.empty_like(dy)
    L.check(L.lib().dfk_spec_augment_bwd(L.ptr(dy), L.ptr(dx), L.ptr(mask), L.ptr(dembed), B, T, C, L.dt(dy),
                                         L.stream()), "spec_augment_bwd")
    return dx


def conv2d_geo(N, H, W, C, k, s, p):
    """dfk_conv2d_geo for a (kh, kw) kernel with stride s and padding p (ints or pairs)."""
    kh, kw = (k, k) if isinstance(k, int) else k
    sh, sw = (s, s) if isinstance(s, int) else s
    ph, pw = (p, p) if isinstance(p, int) else p
    g = L.Conv2dGeo()
    g.N, g.H, g.W, g.C, g.kh, g.kw, g.sh, g.sw, g.ph, g.pw = N, H, W, C, kh, kw, sh, sw, ph, pw
    g.Ho, g.Wo = (H + 2 * ph - kh) // sh + 1, (W + 2 * pw - kw) // sw + 1
    return g


def im2col2d(x, g):
    """x: NHWC view [N, H, W, C] (pixel stride x.stride(2)) -> [N*Ho*Wo, kh*kw*C]."""
    out = torch.empty(g.N * g.Ho * g.Wo, g.kh * g.kw * g.C, device=x.device, dtype=x.dtype)
    L.check(L.lib().dfk_im2col2d(L.ptr(x), x.stride(2), L.ptr(out), g, L.dt(x), L.stream()), "im2col2d")
    return out


def col2im2d(dcols, g, dx, accumulate=False):
    L.check(L.lib().dfk_col2im2d(L.ptr(dcols), L.ptr(dx), dx.stride(2), g, int(accumulate), L.dt(dcols), L.stream()),
            "col2im2d")
    return dx


def bn2d_fwd(x2, y2, gamma, beta, eps, momentum, relu, running_mean=None, running_var=None):
    """Training-mode BatchNorm over the rows of 2-D views x2 -> y2 (+ReLU); returns (mean, rstd)."""
    rows, C = x2.shape
    mean = torch.empty(C, device=x2.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    ws = torch.empty(2 * C, device=x2.device, dtype=torch.float32)
    L.check(L.lib().dfk_bn2d_fwd(L.ptr(x2), x2.stride(0), L.ptr(y2), y2.stride(0), rows, C, L.ptr(gamma), L.ptr(beta),
                                 float(eps), float(momentum), int(relu), L.ptr(mean), L.ptr(rstd),
                                 L.ptr(running_mean), L.ptr(running_var), L.ptr(ws), L.dt(x2), L.stream()), "bn2d_fwd")
    return mean, rstd


def bn2d_apply(x2, y2, mean, rstd, gamma, beta, relu):
    rows, C = x2.shape
    L.check(L.lib().dfk_bn2d_apply(L.ptr(x2), x2.stride(0), L.ptr(y2), y2.stride(0), rows, C, L.ptr(mean), L.ptr(rstd),
                                   L.ptr(gamma), L.ptr(beta), int(relu), L.dt(x2), L.stream()), "bn2d_apply")


def bn2d_bwd(dy2, y2, x2, dx2, mean, rstd, gamma, relu, dgamma, dbeta):
    rows, C = x2.shape
    ws = torch.empty(2 * C, device=x2.device, dtype=torch.float32)
    L.check(L.lib().dfk_bn2d_bwd(L.ptr(dy2), dy2.stride(0), L.ptr(y2), y2.stride(0) if y2 is not None else 0,
                                 L.ptr(x2), x2.stride(0), L.ptr(dx2), dx2.stride(0), rows, C, L.ptr(mean), L.ptr(rstd),
                                 L.ptr(gamma), int(relu), L.ptr(dgamma), L.ptr(dbeta), L.ptr(ws), L.dt(x2),
                                 L.stream()), "bn2d_bwd")


def pool2d_fwd(x, g, mode):
    y = torch.empty(g.N, g.Ho, g.Wo, g.C, device=x.device, dtype=x.dtype)
    L.check(L.lib().dfk_pool2d_fwd(L.ptr(x), x.stride(2), L.ptr(y), y.stride(2), g, int(mode), L.dt(x), L.stream()),
            "pool2d_fwd")
    return y


def pool2d_bwd(x, dy, g, mode, dx=None):
    if dx is None:
        dx = torch.empty(g.N, g.H, g.W, g.C, device=x.device, dtype=x.dtype)
    L.check(L.lib().dfk_pool2d_bwd(L.ptr(x), x.stride(2), L.ptr(dy), dy.stride(2), L.ptr(dx), dx.stride(2), g,
                                   int(mode), 0, L.dt(x), L.stream()), "pool2d_bwd")
    return dx
