"""Media front end on the device: the mel-spectrogram image of
generate_mel_spectrogram (src/utils.py:63-87) and the train-time frame transform of
data/data_process.py:62-69, as HIP kernels (csrc/media.hip) behind plain functions.

The constants the kernels read — the window-folded DFT basis of librosa's STFT and librosa's
Slaney mel filterbank — are built here once per (sr, n_fft, n_mels) in float64 and cast to
float32, as librosa does; they are parameters of the transform, not data.

Parity: librosa, cv2 and PIL are not importable in this image, so the mel image and the
augmentation are pinned to the restatement in oracle/media.py (librosa 0.10 / OpenCV 4 /
torchvision semantics restated from their published algorithms) — parity unpinned against
the libraries themselves."""
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


def draw_augment(frames, device, generator=None, degrees=90.0):
    """Per-frame random parameters of RandomHorizontalFlip / RandomVerticalFlip (p = 0.5) and
    RandomRotation(degrees) (uniform angle in [-degrees, degrees]): (flips int32 [frames], angles fp32 [frames])."""
    g = generator
    hf = (torch.rand(frames, device=device, generator=g) < 0.5).int()
    vf = (torch.rand(frames, device=device, generator=g) < 0.5).int()
    ang = (torch.rand(frames, device=device, generator=g) * 2.0 - 1.0) * degrees
    return (hf | (vf << 1)).int(), ang.float()


def frame_augment(frames_u8, size=(224, 224), flips=None, angles=None, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """uint8 [..., H, W, 3] decoded RGB frames -> fp32 [..., 3, size[1], size[0]]: Resize, flips, rotation,
    ToTensor, Normalize (data_process.py:62-69).  flips / angles: per-frame device tensors (None: off)."""
    *lead, H, W, c3 = frames_u8.shape
    if c3 != 3 or frames_u8.dtype != torch.uint8:
        raise ValueError("frame_augment expects uint8 [..., H, W, 3]")
    x = frames_u8.contiguous()
    n = x.numel() // (H * W * 3)
    ow, oh = size
    out = torch.empty(*lead, 3, oh, ow, device=x.device, dtype=torch.float32)
    fl = flips.to(torch.int32).contiguous() if flips is not None else None
    an = angles.to(torch.float32).contiguous() if angles is not None else None
    for t in (fl, an):
        if t is not None and t.numel() != n:
            raise ValueError("one flip / angle entry per frame")
    L.check(L.lib().dfk_frame_augment(L.ptr(x), n, H, W, oh, ow, L.ptr(fl) if fl is not None else None,
                                      L.ptr(an) if an is not None else None, _f3(mean), _f3(std), L.ptr(out),
                                      L.stream()), "frame_augment")
    return out
