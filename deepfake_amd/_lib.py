"""ctypes binding of libdfk.so (the C ABI declared in include/dfk.h).

The product path has no CPU fallback: importing this module without the
built library, or calling an op with tensors that are not on a HIP device,
raises.  Build with ``python -m deepfake_amd.build``.
"""
import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DFK_LIB") or os.path.join(_HERE, "libdfk.so")   # DFK_LIB: experiment builds (tools/exp_build.sh)

F32, BF16 = 0, 1


class Drop(C.Structure):
    _fields_ = [("rng", C.c_void_p), ("mode", C.c_int32), ("site", C.c_int32), ("p", C.c_float),
                ("group_rows", C.c_int32), ("shared", C.c_int32)]


class View(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("ld", C.c_int64), ("bs0", C.c_int64), ("bs1", C.c_int64),
                ("conv_cg", C.c_int32), ("conv_stride", C.c_int32), ("conv_pad", C.c_int32),
                ("conv_rows", C.c_int32)]


class GemmArgs(C.Structure):
    _fields_ = [("a", View), ("b", View), ("c", C.c_void_p), ("bias", C.c_void_p), ("residual", C.c_void_p),
                ("aux", C.c_void_p), ("ldc", C.c_int64), ("cbs0", C.c_int64), ("cbs1", C.c_int64),
                ("ldr", C.c_int64), ("rbs0", C.c_int64), ("rbs1", C.c_int64), ("ldaux", C.c_int64),
                ("bias_bs1", C.c_int64),
                ("M", C.c_int32), ("N", C.c_int32), ("K", C.c_int32), ("dtype", C.c_int32),
                ("a_kmajor", C.c_int32), ("b_kmajor", C.c_int32), ("c_f32", C.c_int32), ("nz0", C.c_int32),
                ("nz1", C.c_int32), ("splitk", C.c_int32), ("act", C.c_int32), ("atomic", C.c_int32),
                ("beta", C.c_float), ("ws", C.c_void_p), ("rowsum", C.c_void_p), ("drop", Drop),
                ("alpha", C.c_float), ("mx_q", C.c_void_p), ("mx_s", C.c_void_p), ("mx_ldq", C.c_int64),
                ("mx_lds", C.c_int64)]


class MxOperand(C.Structure):
    _fields_ = [("q", C.c_void_p), ("s", C.c_void_p), ("ld", C.c_int64), ("lds", C.c_int64)]


class WattnArgs(C.Structure):
    _fields_ = [("q", C.c_void_p), ("k", C.c_void_p), ("v", C.c_void_p), ("out", C.c_void_p),
                ("rpb", C.c_void_p), ("pad_q", C.c_void_p), ("pad_k", C.c_void_p), ("pad_v", C.c_void_p),
                ("lse", C.c_void_p), ("mask", C.c_void_p), ("mask_nw", C.c_int64),
                ("ld_qkv", C.c_int64), ("ld_out", C.c_int64),
                ("B", C.c_int32), ("D", C.c_int32), ("H", C.c_int32), ("W", C.c_int32),
                ("wd", C.c_int32), ("wh", C.c_int32), ("ww", C.c_int32),
                ("fd", C.c_int32), ("fh", C.c_int32), ("fw", C.c_int32),
                ("sd", C.c_int32), ("sh", C.c_int32), ("sw", C.c_int32),
                ("heads", C.c_int32), ("hd", C.c_int32), ("dtype", C.c_int32), ("scale", C.c_float),
                ("tab", C.c_void_p), ("drop", Drop)]


class WattnBwdArgs(C.Structure):
    _fields_ = [("f", WattnArgs), ("dout", C.c_void_p), ("dq", C.c_void_p), ("dk", C.c_void_p),
                ("dv", C.c_void_p), ("drpb", C.c_void_p), ("dpad_q", C.c_void_p), ("dpad_k", C.c_void_p),
                ("dpad_v", C.c_void_p), ("ld_dqkv", C.c_int64), ("ld_dout", C.c_int64), ("ws", C.c_void_p),
                ("dscore", C.c_void_p)]


class PatchEmbedArgs(C.Structure):
    _fields_ = [("x", C.c_void_p), ("sb", C.c_int64), ("sc", C.c_int64), ("st", C.c_int64), ("sh", C.c_int64),
                ("sw", C.c_int64), ("B", C.c_int32), ("T", C.c_int32), ("H", C.c_int32), ("W", C.c_int32),
                ("C", C.c_int32), ("w", C.c_void_p), ("b", C.c_void_p), ("ln_w", C.c_void_p), ("ln_b", C.c_void_p),
                ("eps", C.c_float), ("out", C.c_void_p), ("mean", C.c_void_p), ("rstd", C.c_void_p),
                ("dw", C.c_void_p), ("db", C.c_void_p), ("dln_w", C.c_void_p), ("dln_b", C.c_void_p)]


class PilResize(C.Structure):
    _fields_ = [("H", C.c_int32), ("W", C.c_int32), ("cin", C.c_int32), ("out_h", C.c_int32), ("out_w", C.c_int32),
                ("xb", C.c_void_p), ("xk", C.c_void_p), ("kx", C.c_int32),
                ("yb", C.c_void_p), ("yk", C.c_void_p), ("ky", C.c_int32)]


class Conv2dGeo(C.Structure):
    _fields_ = [("N", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("C", C.c_int32), ("kh", C.c_int32),
                ("kw", C.c_int32), ("sh", C.c_int32), ("sw", C.c_int32), ("ph", C.c_int32), ("pw", C.c_int32),
                ("Ho", C.c_int32), ("Wo", C.c_int32)]


class Im2colArgs(C.Structure):
    _fields_ = [("sb", C.c_int64), ("sc", C.c_int64), ("st", C.c_int64), ("sh", C.c_int64), ("sw", C.c_int64),
                ("B", C.c_int32), ("cin", C.c_int32), ("T", C.c_int32), ("H", C.c_int32), ("W", C.c_int32),
                ("pd", C.c_int32), ("ph", C.c_int32), ("pw", C.c_int32),
                ("Do", C.c_int32), ("Ho", C.c_int32), ("Wo", C.c_int32)]


# (name, restype, argtypes) for every exported symbol of include/dfk.h
_VP, _I64, _I32, _F = C.c_void_p, C.c_int64, C.c_int32, C.c_float
SIGNATURES = {
    "dfk_gemm": [C.POINTER(GemmArgs), _VP],
    "dfk_gemm_workspace": [C.POINTER(GemmArgs)],
    "dfk_colsum": [_VP, C.c_int, _I64, _I64, _I64, _VP, _VP],
    "dfk_gemm_mx": [C.POINTER(GemmArgs), C.POINTER(MxOperand), C.POINTER(MxOperand), _VP],
    "dfk_mx_quant": [_VP, C.c_int, _I64, _I64, _I64, C.c_int, _VP, _I64, _VP, _VP],
    "dfk_layernorm_fwd": [_VP, _VP, _VP, _VP, _VP, _VP, _I64, _I32, _F, C.c_int, _VP, C.POINTER(Drop), _VP],
    "dfk_layernorm_bwd": [_VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _I64, _I32, C.c_int, C.c_int, _VP,
                          C.POINTER(Drop), _VP, _VP],
    "dfk_layernorm_bwd_workspace": [_I64, _I32],
    "dfk_wattn_fwd": [C.POINTER(WattnArgs), _VP],
    "dfk_wattn_bwd": [C.POINTER(WattnBwdArgs), _VP],
    "dfk_wattn_bwd_workspace": [C.POINTER(WattnArgs)],
    "dfk_wattn_fwd_policy": [C.c_int32, C.c_int64],
    "dfk_wattn_bwd_policy": [C.c_int32, C.c_int32],
    "dfk_wattn_table_workspace": [C.POINTER(WattnArgs)],
    "dfk_wattn_table": [C.POINTER(WattnArgs), _VP],
    "dfk_patch_im2col": [_VP, C.c_int, _VP, C.c_int, C.POINTER(Im2colArgs), _VP],
    "dfk_patch_merge": [_VP, _VP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _VP],
    "dfk_rowmean": [_VP, _VP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _VP],
    "dfk_cast": [_VP, C.c_int, _VP, C.c_int, _I64, _VP],
    "dfk_gelu_bwd": [_VP, _VP, _VP, _I64, C.c_int, _VP],
    "dfk_posconv_wnorm_fwd": [_VP, _VP, C.c_int32, C.c_int32, C.c_int32, _VP, _VP, _VP, _VP, C.c_int, _VP],
    "dfk_posconv_wnorm_bwd": [_VP, _VP, _VP, _VP, C.c_int32, C.c_int32, C.c_int32, _VP, _VP, _VP, _VP],
    "dfk_cosine_qk_fwd": [_VP, _VP, _VP, _F, _I64, C.c_int, C.c_int, C.c_int, _VP],
    "dfk_cosine_qk_bwd": [_VP, _VP, _VP, _VP, _F, _VP, _I64, C.c_int, C.c_int, C.c_int, _VP, _VP],
    "dfk_cpb_bias_fwd": [_VP, _VP, _VP, _VP, _VP, _I32, _I32, _I32, _VP],
    "dfk_cpb_bias_bwd": [_VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _I32, _I32, _I32, _VP],
    "dfk_cpb_bias_fwd_many": [_VP, _I32, _I32, _VP, _VP],
    "dfk_cpb_bias_bwd_many": [_VP, _I32, _I32, _VP, _VP, _VP],
    "dfk_w2v_conv0_fwd": [_VP, _I64, _I64, _VP, _VP, _VP, _F, _VP, _VP, C.c_int, _VP, _VP],
    "dfk_w2v_conv0_fwd_workspace": [_I64, _I64],
    "dfk_w2v_conv0_bwd": [_VP, _I64, _I64, _VP, _VP, _VP, _F, _VP, _VP, C.c_int, _VP, _I64, _VP, _VP, _VP, _VP],
    "dfk_w2v_conv0_bwd_workspace": [_I64, _I64],
    "dfk_sgd_step_runs": [_VP, _VP, _VP, _VP, _VP, C.c_int32, _VP, _F, _F, _F, _F, _VP, _VP],
    "dfk_sgd_step": [_VP, _VP, _VP, _VP, _I64, _VP, _F, _F, _F, C.c_int, _VP, _F, _VP, _VP],
    "dfk_im2col2d": [_VP, _I64, _VP, C.POINTER(Conv2dGeo), C.c_int, _VP],
    "dfk_col2im2d": [_VP, _VP, _I64, C.POINTER(Conv2dGeo), C.c_int, C.c_int, _VP],
    "dfk_bn2d_fwd": [_VP, _I64, _VP, _I64, _I64, _I32, _VP, _VP, _F, _F, C.c_int, _VP, _VP, _VP, _VP, _VP, C.c_int,
                     _VP],
    "dfk_bn2d_apply": [_VP, _I64, _VP, _I64, _I64, _I32, _VP, _VP, _VP, _VP, C.c_int, C.c_int, _VP],
    "dfk_bn2d_bwd": [_VP, _I64, _VP, _I64, _VP, _I64, _VP, _I64, _I64, _I32, _VP, _VP, _VP, C.c_int, _VP, _VP, _VP,
                     C.c_int, _VP],
    "dfk_pool2d_fwd": [_VP, _I64, _VP, _I64, C.POINTER(Conv2dGeo), C.c_int, C.c_int, _VP],
    "dfk_pool2d_bwd": [_VP, _I64, _VP, _I64, _VP, _I64, C.POINTER(Conv2dGeo), C.c_int, C.c_int, C.c_int, _VP],
    "dfk_dropout": [_VP, _VP, _I64, _I32, _I64, C.POINTER(Drop), C.c_int, _VP],
    "dfk_bernoulli_flags": [C.POINTER(Drop), _I32, _VP, _VP],
    "dfk_mel_workspace": [_I64, _I64, _I32, _I32, _I32],
    "dfk_mel_image": [_VP, _I64, _I64, _VP, _VP, _I32, _I32, _I32, _I32, _I32, _VP, _I64, _VP, _VP],
    "dfk_gray_normalize": [_VP, _VP, _I64, _I32, _I32, C.POINTER(C.c_float), C.POINTER(C.c_float), _VP],
    "dfk_frame_augment": [_VP, _I64, C.POINTER(PilResize), _VP, _VP, C.POINTER(C.c_float), C.POINTER(C.c_float),
                          _VP, _VP, _VP],
    "dfk_layerdrop_flags": [C.POINTER(Drop), _I32, _VP, _VP, _VP],
    "dfk_layer_select": [_VP, _VP, _VP, _VP, _VP, C.c_int64, _VP],
    "dfk_spec_augment_fwd": [_VP, _VP, _VP, _VP, _I32, _I32, _I32, _F, _I32, _I32, C.POINTER(Drop), C.c_int, _VP],
    "dfk_spec_augment_bwd": [_VP, _VP, _VP, _VP, _I32, _I32, _I32, C.c_int, _VP],
    "dfk_frame_normalize": [_VP, _VP, _I64, _I32, _I32, C.POINTER(C.c_float), C.POINTER(C.c_float), _VP],
    "dfk_wave_normalize": [_VP, _VP, _I64, _I64, _F, _VP],
    "dfk_patch_embed_fwd": [C.POINTER(PatchEmbedArgs), _VP],
    "dfk_patch_embed_bwd": [C.POINTER(PatchEmbedArgs), _VP, _VP],
}

_lib = None
RESTYPES = {"dfk_mel_workspace": _I64, "dfk_w2v_conv0_bwd_workspace": _I64, "dfk_w2v_conv0_fwd_workspace": _I64, "dfk_layernorm_bwd_workspace": _I64, "dfk_wattn_bwd_workspace": _I64, "dfk_wattn_table_workspace": _I64, "dfk_gemm_workspace": _I64}


def lib():
    """Load libdfk.so once; raise (never fall back) if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"deepfake_amd: {LIB_PATH} not built — run `python -m deepfake_amd.build`")
        L = C.CDLL(LIB_PATH)
        for name, argt in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = RESTYPES.get(name, C.c_int)
            fn.argtypes = argt
        _lib = L
    return _lib


def exported_symbols():
    return list(SIGNATURES)


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"deepfake_amd: {what} failed (rc={rc}{' EINVAL' if rc == -1 else ''})")


def ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("deepfake_amd: tensors must be on the HIP device (no CPU fallback)")
    return C.c_void_p(t.data_ptr())


def drop(spec, device):
    """ctypes dfk_drop for a rng.Drop spec tuple (mode, site, p, group_rows, shared), or None."""
    if spec is None:
        return None
    from . import rng
    d = Drop()
    d.rng = rng.state(device).data_ptr()
    d.mode, d.site, d.p, d.group_rows, d.shared = int(spec[0]), int(spec[1]), float(spec[2]), int(spec[3]), \
        int(spec[4])
    return d


def dt(t):
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float32:
        return F32
    raise TypeError(f"deepfake_amd: unsupported dtype {t.dtype}")
