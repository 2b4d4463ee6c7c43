"""Media front end on the device: the mel-spectrogram image of
generate_mel_spectrogram (src/utils.py:63-87) and the train-time frame transform of
data/data_process.py:62-69, as HIP kernels (csrc/media.hip) behind plain functions.

The constants the kernels read — the window-folded DFT basis of librosa's STFT and librosa's
Slaney mel filterbank — are built here once per (sr, n_fft, n_mels) in float64 and cast to
float32, as librosa does; they are parameters of the transform, not data.

Parity: the frame / mel-image transform follows PIL 12.2 (importable here), as the reference applies
torchvision's transforms to PIL images: pinned bit for bit to PIL fixtures (tests/golden/pil_frames.npz, written
by tests/golden/make_pil_fixtures.py).  librosa and cv2 are absent, so the mel-spectrogram image stays pinned to
the restatement in oracle/media.py (librosa 0.10 / OpenCV 4 semantics from their published algorithms) — parity
unpinned against those libraries."""
import ctypes
import functools
import math

import numpy as np
import torch

from . import _lib as L

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _hz_to_mel(f):
    """Slaney mel scale (librosa.hz_to_mel, htk=False)."""
    f = np.asanyarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, f / f_sp)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


@functools.lru_cache(maxsize=8)
def mel_filterbank(sr=22050, n_fft=2048, n_mels=128, fmin=0.0, fmax=None):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk=False, norm='slaney') -> float32 [n_mels, 1+n_fft/2]."""
    fmax = sr / 2.0 if fmax is None else fmax
    fftfreqs = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0.0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


@functools.lru_cache(maxsize=8)
def stft_basis(n_fft=2048):
    """Window-folded real DFT basis [n_fft, ld] (ld = 2 (n_fft/2+1) rounded up to 4): column f = w[n] cos(2 pi f n / N),
    column nbin + f = -w[n] sin(...), w = periodic Hann (librosa's get_window('hann', fftbins=True)), so that
    frames @ basis gives Re | Im of np.fft.rfft(w * frame)."""
    nbin = n_fft // 2 + 1
    ld = (2 * nbin + 3) // 4 * 4
    n = np.arange(n_fft)
    w = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / n_fft)
    k = np.outer(n, np.arange(nbin)) % n_fft          # exact phase index before the float conversion
    ang = 2.0 * np.pi * k / n_fft
    b = np.zeros((n_fft, ld))
    b[:, :nbin] = w[:, None] * np.cos(ang)
    b[:, nbin:2 * nbin] = -w[:, None] * np.sin(ang)
    return b.astype(np.float32)


_DEV_CONST = {}


def _const(key, make, device):
    k = (key, str(device))
    t = _DEV_CONST.get(k)
    if t is None:
        t = torch.from_numpy(make()).to(device)
        _DEV_CONST[k] = t
    return t


def mel_image(wave, sr=22050, n_fft=2048, hop=512, n_mels=128, size=(224, 224)):
    """wave fp32 [B, S] (device, at `sr`) -> uint8 [B, size[1], size[0]] mel-spectrogram images
    (generate_mel_spectrogram, src/utils.py:63-87; the reference's fmax argument is unused there)."""
    if not wave.is_cuda:
        raise RuntimeError("mel_image: device tensors only (no CPU fallback)")
    x = wave.float().contiguous()
    B, S = x.shape
    basis = _const(("basis", n_fft), lambda: stft_basis(n_fft), x.device)
    fb = _const(("fb", sr, n_fft, n_mels), lambda: mel_filterbank(sr, n_fft, n_mels), x.device)
    nbytes = L.lib().dfk_mel_workspace(B, S, n_fft, hop, n_mels)
    if nbytes < 0:
        raise RuntimeError("dfk_mel_workspace: invalid arguments")
    ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
    ow, oh = size
    out = torch.empty(B, oh, ow, dtype=torch.uint8, device=x.device)
    L.check(L.lib().dfk_mel_image(L.ptr(x), B, S, L.ptr(basis), L.ptr(fb), n_fft, hop, n_mels, oh, ow, L.ptr(ws),
                                  nbytes, L.ptr(out), L.stream()), "mel_image")
    return out


def _f3(v):
    return (ctypes.c_float * 3)(*v)


def gray_normalize(img_u8, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """uint8 [..., H, W] gray images -> fp32 [..., 3, H, W] (convert('RGB') + ToTensor + Normalize)."""
    *lead, H, W = img_u8.shape
    x = img_u8.contiguous()
    out = torch.empty(*lead, 3, H, W, device=x.device, dtype=torch.float32)
    L.check(L.lib().dfk_gray_normalize(L.ptr(x), L.ptr(out), x.numel() // (H * W), H, W, _f3(mean), _f3(std),
                                       L.stream()), "gray_normalize")
    return out


def pil_bilinear_coeffs(in_size, out_size):
    """PIL's Image.resize(BILINEAR) coefficients along one axis (libImaging/Resample.c precompute_coeffs with the
    triangle filter, support 1 scaled by max(1, in/out), then normalize_coeffs_8bpc's 22-bit fixed point):
    (bounds int32 [out, 2] = (first source index, tap count), coeffs int32 [out, ksize], ksize)."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int32)
    kk = np.zeros((out_size, ksize), dtype=np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)          # C (int): truncation toward zero
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            v = 1.0 - t if t < 1.0 else 0.0
            w.append(v)
            ww += v
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + k * (1 << 22)) if k < 0 else int(0.5 + k * (1 << 22))
        bounds[xx] = (xmin, xmax)
    return bounds, kk, ksize


def pil_rotate_fixed(angle, w, h):
    """Image.rotate(angle, NEAREST, expand=False) of a w x h image as PIL 12 runs it: the inverse affine matrix
    built in Image.rotate (angle % 360, cos / sin rounded to 15 decimals, rotation about (w/2, h/2)), then
    libImaging affine_fixed's 16.16 fixed point with the pixel-centre offset folded into the translation.
    Returns 8 int32 {on, a0, a1, a2, a3, a4, a5, 0}; on = 0 for the copy fast path (angle % 360 == 0).  The 180 /
    90 / 270 transpose fast paths give the same map as this affine (exact rounded cos / sin)."""
    angle = angle % 360.0
    if angle == 0:
        return [0] * 8
    cx, cy = w / 2, h / 2
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0, round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    m[2] = m[0] * -cx + m[1] * -cy + m[2] + cx
    m[5] = m[3] * -cx + m[4] * -cy + m[5] + cy

    def fix(v):
        return math.floor(v * 65536.0 + 0.5)
    return [1, fix(m[0]), fix(m[1]), fix(m[2] + m[1] * 0.5 + m[0] * 0.5), fix(m[3]), fix(m[4]),
            fix(m[5] + m[4] * 0.5 + m[3] * 0.5), 0]


@functools.lru_cache(maxsize=16)
def _pil_axis(in_size, out_size):
    b, k, ks = pil_bilinear_coeffs(in_size, out_size)
    return b, k, ks


def eval_size(H, W, short=224):
    """torchvision T.Resize(int) output size (h, w): the shorter side to `short`, the longer scaled and truncated."""
    if W <= H:
        return int(short * H / W), short
    return short, int(short * W / H)


def draw_augment(frames, generator=None, degrees=90.0):
    """Per-frame parameters of T.RandomHorizontalFlip, T.RandomVerticalFlip (p = 0.5) and T.RandomRotation(90),
    drawn on the CPU in the order the reference's Compose draws them for each frame (torch.rand(1) < 0.5,
    torch.rand(1) < 0.5, torch.empty(1).uniform_(-90, 90)): (flips int32 [frames] (bit 0 horizontal, bit 1
    vertical), angles: list of Python floats).  One batched draw of [frames, 3] uniforms: the CPU generator
    hands them out in the same sequence as the per-frame scalar calls, and uniform_(a, b) on one float is
    float32(double(u) * (b - a) + a) of the same 24-bit draw, so flips, angles and the generator's state afterwards
    are identical to the scalar loop (tests/test_media_oracle.py pins this)."""
    u = torch.rand(frames, 3, generator=generator)
    flips = ((u[:, 0] < 0.5).int() | ((u[:, 1] < 0.5).int() << 1)).to(torch.int32)
    angles = (u[:, 2].double() * (2.0 * degrees) - degrees).float()
    return flips, angles.tolist()


def frame_augment(frames_u8, size=(224, 224), flips=None, angles=None, mean=IMAGENET_MEAN, std=IMAGENET_STD,
                  grey=False):
    """uint8 [..., H, W, 3] decoded RGB frames (or, with grey=True, [..., H, W] grey images) on the device -> fp32
    [..., 3, size[1], size[0]]: PIL Resize, flips, rotation, ToTensor, Normalize (data_process.py:55-69 on PIL
    images).  flips: int tensor [frames] (None: none); angles: per-frame rotation angles in degrees (host floats,
    None: none)."""
    x = frames_u8
    if x.dtype != torch.uint8:
        raise ValueError("frame_augment expects uint8 frames")
    if grey and x.dim() < 2:
        raise ValueError("grey frame_augment expects [..., H, W]")
    if not grey and (x.dim() < 3 or x.shape[-1] != 3):
        raise ValueError("frame_augment expects RGB frames [..., H, W, 3] (grey=True for [..., H, W])")
    *lead, H, W = (x.shape if grey else x.shape[:-1])
    cin = 1 if grey else 3
    x = x.contiguous()
    n = x.numel() // (H * W * cin)
    ow, oh = size
    dev = x.device
    xb, xk, kx = _pil_axis(W, ow)
    yb, yk, ky = _pil_axis(H, oh)
    cxb, cxk = _const(("pilx", W, ow, "b"), lambda: xb, dev), _const(("pilx", W, ow, "k"), lambda: xk, dev)
    cyb, cyk = _const(("pily", H, oh, "b"), lambda: yb, dev), _const(("pily", H, oh, "k"), lambda: yk, dev)
    r = L.PilResize()
    r.H, r.W, r.cin, r.out_h, r.out_w = H, W, cin, oh, ow
    r.xb, r.xk, r.kx = cxb.data_ptr(), cxk.data_ptr(), kx
    r.yb, r.yk, r.ky = cyb.data_ptr(), cyk.data_ptr(), ky
    fl = flips.to(device=dev, dtype=torch.int32).contiguous() if flips is not None else None
    aff = None
    if angles is not None:
        if len(angles) != n:
            raise ValueError("one angle per frame")
        aff = torch.tensor([pil_rotate_fixed(float(a), ow, oh) for a in angles], dtype=torch.int32).to(dev)
    if fl is not None and fl.numel() != n:
        raise ValueError("one flip entry per frame")
    tmp = torch.empty(n * H * ow * cin, dtype=torch.uint8, device=dev)
    out = torch.empty(*lead, 3, oh, ow, device=dev, dtype=torch.float32)
    L.check(L.lib().dfk_frame_augment(L.ptr(x), n, r, L.ptr(fl) if fl is not None else None,
                                      L.ptr(aff) if aff is not None else None, _f3(mean), _f3(std), L.ptr(tmp),
                                      L.ptr(out), L.stream()), "frame_augment")
    return out
