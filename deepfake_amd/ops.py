"""The native ops as PyTorch operators: the ``dfk`` library (torch.library — the Python registration of
TORCH_LIBRARY(dfk, m)), so the hot path is reachable as ``torch.ops.dfk.*`` by any torch
program, traceable by torch.compile / torch.export (every op has a fake implementation for shape
propagation) and differentiable through registered backward formulas.

    import deepfake_amd.ops
    y = torch.ops.dfk.linear(x, w, b)                      # nn.Linear (src/utils.py:249-251)
    y, mean, rstd = torch.ops.dfk.layer_norm(x, w, b, 1e-5)
    o, lse, tab = torch.ops.dfk.window_attention(qkv, rpb, pad, [B,D,H,W], window, full_window, shift,
                                                 heads, hd, scale)

Each op calls the same C ABI entry point as the model's modules (include/dfk.h) on the current HIP stream;
there is no CPU kernel (a CPU tensor raises, as everywhere in the product).  The model code keeps calling the
kernels through deepfake_amd.functional, whose direct-gradient protocol (weight gradients accumulated straight
into the flat gradient buffer) has no torch.library equivalent; these operators are the interface for other
callers."""
import torch

from . import _lib as L
from . import kernels as K

LIB = "dfk"


def _need_gpu(t):
    if not t.is_cuda:
        raise RuntimeError(f"dfk ops run on the GPU only (got a {t.device} tensor); there is no CPU kernel")

# --------------------------------------------------------------------------------------------- linear
@torch.library.custom_op("dfk::linear", mutates_args=())
def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """y = x w^T + b on dfk_gemm (bf16 / fp32 MFMA); x [M, K], w [N, K]."""
    _need_gpu(x)
    return K.linear(x.contiguous(), w.contiguous(), b.contiguous() if b is not None else None)


@linear.register_fake
def _(x, w, b=None):
    return x.new_empty(x.shape[0], w.shape[0])


@torch.library.custom_op("dfk::linear_dx", mutates_args=())
def linear_dx(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    _need_gpu(dy)
    return K.linear_dx(dy.contiguous(), w.contiguous())


@linear_dx.register_fake
def _(dy, w):
    return dy.new_empty(dy.shape[0], w.shape[1])


@torch.library.custom_op("dfk::linear_dw", mutates_args=())
def linear_dw(dy: torch.Tensor, x: torch.Tensor) -> list[torch.Tensor]:
    """(dW [N, K] fp32, db [N] fp32) of y = x w^T + b."""
    _need_gpu(dy)
    dw = torch.zeros(dy.shape[1], x.shape[1], device=dy.device, dtype=torch.float32)
    db = torch.zeros(dy.shape[1], device=dy.device, dtype=torch.float32)
    K.linear_dw(dy.contiguous(), x.contiguous(), dw, db)
    return [dw, db]


@linear_dw.register_fake
def _(dy, x):
    return [dy.new_empty(dy.shape[1], x.shape[1], dtype=torch.float32),
            dy.new_empty(dy.shape[1], dtype=torch.float32)]


def _linear_setup(ctx, inputs, output):
    x, w, b = inputs
    ctx.save_for_backward(x, w)
    ctx.has_b = b is not None


def _linear_bwd(ctx, dy):
    x, w = ctx.saved_tensors
    dx = torch.ops.dfk.linear_dx(dy, w)
    dw, db = torch.ops.dfk.linear_dw(dy, x)
    return dx, dw.to(w.dtype), (db.to(w.dtype) if ctx.has_b else None)


linear.register_autograd(_linear_bwd, setup_context=_linear_setup)


# ----------------------------------------------------------------------------------------- layer_norm
@torch.library.custom_op("dfk::layer_norm", mutates_args=())
def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> list[torch.Tensor]:
    """(y, mean fp32, rstd fp32) of nn.LayerNorm over the last dim of a [rows, C] tensor."""
    _need_gpu(x)
    y, mean, rstd = K.layernorm_fwd(x.contiguous(), w.contiguous(), b.contiguous(), eps)
    return [y, mean, rstd]


@layer_norm.register_fake
def _(x, w, b, eps):
    return [torch.empty_like(x), x.new_empty(x.shape[0], dtype=torch.float32),
            x.new_empty(x.shape[0], dtype=torch.float32)]


@torch.library.custom_op("dfk::layer_norm_bwd", mutates_args=())
def layer_norm_bwd(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, mean: torch.Tensor,
                   rstd: torch.Tensor) -> list[torch.Tensor]:
    _need_gpu(x)
    dw = torch.zeros(w.shape[0], device=x.device, dtype=torch.float32)
    db = torch.zeros(w.shape[0], device=x.device, dtype=torch.float32)
    dx = K.layernorm_bwd(dy.contiguous(), x.contiguous(), w.contiguous(), mean, rstd, dw, db)
    return [dx, dw, db]


@layer_norm_bwd.register_fake
def _(dy, x, w, mean, rstd):
    return [torch.empty_like(x), w.new_empty(w.shape[0], dtype=torch.float32),
            w.new_empty(w.shape[0], dtype=torch.float32)]


def _ln_setup(ctx, inputs, output):
    x, w, b, eps = inputs
    ctx.save_for_backward(x, w, output[1], output[2])


def _ln_bwd(ctx, grads):
    dy = grads[0]
    x, w, mean, rstd = ctx.saved_tensors
    dx, dw, db = torch.ops.dfk.layer_norm_bwd(dy, x, w, mean, rstd)
    return dx, dw.to(w.dtype), db.to(w.dtype), None


layer_norm.register_autograd(_ln_bwd, setup_context=_ln_setup)


# -------------------------------------------------------------------------------------- window_attention
def _pads(pad, C):
    return (pad[:C], pad[C:2 * C], pad[2 * C:]) if pad is not None else None


@torch.library.custom_op("dfk::window_attention", mutates_args=())
def window_attention(qkv: torch.Tensor, rpb: torch.Tensor | None, pad: torch.Tensor | None, dims: list[int],
                     window: list[int], full_window: list[int], shift: list[int], heads: int, hd: int,
                     scale: float) -> list[torch.Tensor]:
    """WindowAttention3D core with forward_part1's pad / roll / window partition and their inverses
    (video_swin_transformer.py:142-173, :224-252) on a token-major qkv [B*D*H*W, 3C]: (out [rows, C], lse, bias
    tiles).  rpb [(2Wd-1)(2Wh-1)(2Ww-1), heads] (None: no position bias); pad [3C]: q|k|v of a padded token (the
    qkv Linear's bias, since the reference zero-pads x before the projection; None: zero)."""
    _need_gpu(qkv)
    C = heads * hd
    q = qkv.contiguous()
    rpb_f = rpb.float().contiguous() if rpb is not None else None
    out, lse, tab = K.wattn_fwd(q, q[:, C:], q[:, 2 * C:], 3 * C, dims, window, full_window, shift, heads, hd, scale,
                                rpb=rpb_f, pads=_pads(pad.to(q.dtype).contiguous() if pad is not None else None, C),
                                return_table=True)
    if tab is None:
        tab = q.new_empty(0, dtype=torch.float32)
    return [out, lse, tab]


def _table_numel(dims, window, full_window, shift, heads, hd, has_rpb, dtype):
    """Float count of the bias tiles dfk_wattn_table builds for this geometry (0 without rpb and shift)."""
    a = L.WattnArgs()
    a.B, a.D, a.H, a.W = (int(d) for d in dims)
    a.wd, a.wh, a.ww = (int(w) for w in window)
    a.fd, a.fh, a.fw = (int(w) for w in full_window)
    a.sd, a.sh, a.sw = (int(s) for s in shift)
    a.heads, a.hd = int(heads), int(hd)
    a.dtype = L.BF16 if dtype == torch.bfloat16 else L.F32
    a.ld_qkv, a.ld_out = 3 * a.heads * a.hd, a.heads * a.hd
    a.q = a.k = a.v = a.out = 1              # the size query checks presence only and dereferences nothing
    a.rpb = 1 if has_rpb else None
    nbytes = L.lib().dfk_wattn_table_workspace(a)
    if nbytes < 0:
        raise RuntimeError("dfk_wattn_table_workspace: invalid arguments")
    return nbytes // 4


@window_attention.register_fake
def _(qkv, rpb, pad, dims, window, full_window, shift, heads, hd, scale):
    nW, N, Np = K.window_geometry(dims, window)
    ntab = _table_numel(dims, window, full_window, shift, heads, hd, rpb is not None, qkv.dtype)
    return [qkv.new_empty(qkv.shape[0], heads * hd), qkv.new_empty(dims[0] * nW * heads, Np, dtype=torch.float32),
            qkv.new_empty(ntab, dtype=torch.float32)]


@torch.library.custom_op("dfk::window_attention_bwd", mutates_args=())
def window_attention_bwd(dout: torch.Tensor, qkv: torch.Tensor, out: torch.Tensor, lse: torch.Tensor,
                         tab: torch.Tensor, rpb: torch.Tensor | None, pad: torch.Tensor | None, dims: list[int],
                         window: list[int], full_window: list[int], shift: list[int], heads: int, hd: int,
                         scale: float) -> list[torch.Tensor]:
    """(dqkv, drpb fp32 (empty without rpb), dpad fp32 [3C] (empty without pad))."""
    _need_gpu(qkv)
    C = heads * hd
    q = qkv.contiguous()
    dqkv = torch.empty_like(q)
    rpb_f = rpb.float().contiguous() if rpb is not None else None
    drpb = torch.zeros_like(rpb_f) if rpb is not None else q.new_zeros(0, dtype=torch.float32)
    dpad = q.new_zeros(3 * C if pad is not None else 0, dtype=torch.float32)
    K.wattn_bwd((q, q[:, C:], q[:, 2 * C:], out, lse, 3 * C, dims, window, full_window, shift, heads, hd, scale, rpb_f,
                 _pads(pad.to(q.dtype).contiguous() if pad is not None else None, C)), dout.contiguous(), dqkv,
                dqkv[:, C:], dqkv[:, 2 * C:], 3 * C, drpb=drpb if rpb is not None else None,
                dpads=_pads(dpad, C), tab=tab if tab.numel() else None)
    return [dqkv, drpb, dpad]


@window_attention_bwd.register_fake
def _(dout, qkv, out, lse, tab, rpb, pad, dims, window, full_window, shift, heads, hd, scale):
    C = heads * hd
    return [torch.empty_like(qkv), qkv.new_empty(rpb.shape if rpb is not None else (0,), dtype=torch.float32),
            qkv.new_empty(3 * C if pad is not None else 0, dtype=torch.float32)]


def _wa_setup(ctx, inputs, output):
    qkv, rpb, pad, dims, window, full_window, shift, heads, hd, scale = inputs
    ctx.save_for_backward(qkv, output[0], output[1], output[2], rpb, pad)
    ctx.geo = (list(dims), list(window), list(full_window), list(shift), heads, hd, scale)


def _wa_bwd(ctx, grads):
    qkv, out, lse, tab, rpb, pad = ctx.saved_tensors
    dqkv, drpb, dpad = torch.ops.dfk.window_attention_bwd(grads[0], qkv, out, lse, tab, rpb, pad, *ctx.geo)
    return (dqkv, drpb.to(rpb.dtype) if rpb is not None else None,
            dpad.to(pad.dtype) if pad is not None else None) + (None,) * 7


window_attention.register_autograd(_wa_bwd, setup_context=_wa_setup)


# ------------------------------------------------------------------------------------ media front end
@torch.library.custom_op("dfk::mel_image", mutates_args=())
def mel_image(wave: torch.Tensor, sr: int = 22050, n_fft: int = 2048, hop: int = 512, n_mels: int = 128,
              out_h: int = 224, out_w: int = 224) -> torch.Tensor:
    """generate_mel_spectrogram (src/utils.py:63-87) from a device waveform [B, S]: uint8 [B, out_h, out_w]."""
    _need_gpu(wave)
    from . import media
    return media.mel_image(wave, sr, n_fft, hop, n_mels, (out_w, out_h))


@mel_image.register_fake
def _(wave, sr=22050, n_fft=2048, hop=512, n_mels=128, out_h=224, out_w=224):
    return wave.new_empty(wave.shape[0], out_h, out_w, dtype=torch.uint8)


@torch.library.custom_op("dfk::frame_augment", mutates_args=())
def frame_augment(frames: torch.Tensor, flips: torch.Tensor | None, angles: torch.Tensor | None, out_h: int = 224,
                  out_w: int = 224) -> torch.Tensor:
    """The training frame transform (data_process.py:62-69, PIL semantics) of uint8 [..., H, W, 3] frames; angles
    (degrees, one per frame) are read on the host (the rotation's fixed-point matrices are built there, as PIL
    builds them)."""
    _need_gpu(frames)
    from . import media
    ang = [float(a) for a in angles.detach().cpu().reshape(-1)] if angles is not None else None
    return media.frame_augment(frames, (out_w, out_h), flips, ang)


@frame_augment.register_fake
def _(frames, flips, angles, out_h=224, out_w=224):
    return frames.new_empty(*frames.shape[:-3], 3, out_h, out_w, dtype=torch.float32)


OPS = ("linear", "linear_dx", "linear_dw", "layer_norm", "layer_norm_bwd", "window_attention",
       "window_attention_bwd", "mel_image", "frame_augment")
