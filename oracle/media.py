"""Oracle (test infrastructure only) for the f2 media front end: numpy restatement of
generate_mel_spectrogram (/root/reference/src/utils.py:63-87) and of the train-time frame
transform (/root/reference/data/data_process.py:62-69).

The arithmetic lives in libraries the reference imports but this image lacks (librosa, cv2,
PIL/torchvision), so it is restated from their published algorithms:
  librosa 0.10: feature.melspectrogram (stft: periodic Hann, center=True, pad_mode='constant',
      power 2; filters.mel: Slaney scale, norm='slaney'), power_to_db(ref=np.max, amin=1e-10,
      top_db=80);
  OpenCV 4: normalize(NORM_MINMAX, 0, 255) (double scale / shift), astype(uint8) truncation,
      resize(INTER_LINEAR) on uint8 (11-bit fixed-point coefficients, 22-bit rounding shift);
  PIL 12.2 (the frame / mel-image transform: torchvision's transforms run on PIL images in the reference,
      src/utils.py:32-33, data_process.py:55-69,162): Image.resize(BILINEAR) (libImaging/Resample.c: triangle
      filter with support scaled by the downscale factor, 22-bit fixed-point coefficients, width pass then height
      pass, each into uint8), Image.rotate(NEAREST, fill 0) (Image.rotate's inverse matrix, affine_fixed's 16.16
      fixed-point walk), transpose flips.
The PIL restatement is pinned bit for bit to fixtures written with PIL itself (tests/golden/pil_frames.npz,
tests/golden/make_pil_fixtures.py).  librosa / cv2 are absent: the mel-spectrogram stage is PARITY UNPINNED
against them; its STFT is checked against torch.stft.
"""
import math

import numpy as np


def hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp, min_log_hz, logstep = 200.0 / 3, 1000.0, math.log(6.4) / 27.0
    mel = f / f_sp
    hi = f >= min_log_hz
    mel[hi] = min_log_hz / f_sp + np.log(f[hi] / min_log_hz) / logstep
    return mel


def mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp, min_log_hz, logstep = 200.0 / 3, 1000.0, math.log(6.4) / 27.0
    f = f_sp * m
    hi = m >= min_log_hz / f_sp
    f[hi] = min_log_hz * np.exp(logstep * (m[hi] - min_log_hz / f_sp))
    return f


def mel_filters(sr, n_fft, n_mels):
    fft = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(np.array([0.0]))[0], hz_to_mel(np.array([sr / 2.0]))[0], n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fft[None, :]
    w = np.zeros((n_mels, len(fft)))
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


def stft_power(y, n_fft=2048, hop=512):
    """|rfft(hann * frame)|^2 of the center-zero-padded signal: [1 + n_fft/2, 1 + len(y)//hop] (float64)."""
    y = np.asarray(y, dtype=np.float64)
    yp = np.pad(y, (n_fft // 2, n_fft // 2))
    T = 1 + len(y) // hop
    idx = np.arange(n_fft)[None, :] + hop * np.arange(T)[:, None]
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft)
    X = np.fft.rfft(yp[idx] * w[None, :], axis=1)
    return (np.abs(X) ** 2).T


def mel_db_uint8(y, sr=22050, n_fft=2048, hop=512, n_mels=128):
    """melspectrogram -> power_to_db(ref=max) -> cv2 min-max -> uint8, the [n_mels, T] image before the resize."""
    S = (mel_filters(sr, n_fft, n_mels).astype(np.float64) @ stft_power(y, n_fft, hop)).astype(np.float32)
    amin = np.float32(1e-10)
    db = np.float32(10.0) * np.log10(np.maximum(amin, S))
    db -= np.float32(10.0) * np.log10(np.maximum(amin, S.max()))
    db = np.maximum(db, db.max() - np.float32(80.0))
    lo, hi = float(db.min()), float(db.max())
    scale = 255.0 / (hi - lo) if hi > lo else 0.0
    q = (db.astype(np.float64) * scale - lo * scale).astype(np.float32)
    return np.clip(q, 0, 255).astype(np.uint8)


def _cv_taps(dn, sn):
    scale = sn / dn
    out = []
    for d in range(dn):
        fx = np.float32((d + 0.5) * scale - 0.5)
        sx = int(np.floor(fx))
        fx = np.float32(fx - np.float32(sx))
        if sx < 0:
            fx, sx = np.float32(0), 0
        if sx >= sn - 1:
            fx, sx = np.float32(0), sn - 1
        a0 = int(np.rint(np.float32(1.0 - fx) * np.float32(2048.0)))
        a1 = int(np.rint(fx * np.float32(2048.0)))
        out.append((sx, min(sx + 1, sn - 1), a0, a1))
    return out


def cv_resize_linear_u8(img, size):
    """cv2.resize(img, size=(w, h), interpolation=INTER_LINEAR) for uint8 (fixed point, 11-bit weights)."""
    h_in, w_in = img.shape
    ow, oh = size
    xt, yt = _cv_taps(ow, w_in), _cv_taps(oh, h_in)
    im = img.astype(np.int64)
    out = np.zeros((oh, ow), dtype=np.uint8)
    for dy, (y0, y1, b0, b1) in enumerate(yt):
        for dx, (x0, x1, a0, a1) in enumerate(xt):
            r0 = im[y0, x0] * a0 + im[y0, x1] * a1
            r1 = im[y1, x0] * a0 + im[y1, x1] * a1
            out[dy, dx] = min(max((b0 * r0 + b1 * r1 + (1 << 21)) >> 22, 0), 255)
    return out


def mel_image(y, sr=22050, n_fft=2048, hop=512, n_mels=128, size=(224, 224)):
    """generate_mel_spectrogram from the decoded waveform on (the file I/O and the resampling excluded)."""
    return cv_resize_linear_u8(mel_db_uint8(y, sr, n_fft, hop, n_mels), size)


# ---------------------------------------------------------------- PIL 12.2 frame transform
def pil_coeffs(in_size, out_size):
    """libImaging/Resample.c precompute_coeffs (BILINEAR: triangle, support 1) + normalize_coeffs_8bpc."""
    scale = float(in_size) / out_size
    fscale = max(scale, 1.0)
    support = fscale
    taps = []
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [max(0.0, 1.0 - abs((x + xmin - center + 0.5) / fscale)) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        k = [(v / ww if ww != 0.0 else v) for v in w]
        taps.append((xmin, [int(-0.5 + v * (1 << 22)) if v < 0 else int(0.5 + v * (1 << 22)) for v in k]))
    return taps


def _pass(img, taps, axis):
    """One separable pass over `axis` of a uint8 [h, w, c] image (22-bit rounding, clip to uint8)."""
    im = np.moveaxis(img.astype(np.int64), axis, 0)
    out = np.empty((len(taps),) + im.shape[1:], dtype=np.uint8)
    for o, (x0, k) in enumerate(taps):
        acc = np.full(im.shape[1:], 1 << 21, dtype=np.int64)
        for t, kv in enumerate(k):
            acc += im[x0 + t] * kv
        out[o] = np.clip(acc >> 22, 0, 255)
    return np.moveaxis(out, 0, axis)


def pil_resize_bilinear(img, size):
    """Image.resize((w, h), BILINEAR) of a uint8 [h, w, c] image: width pass, then height pass."""
    ow, oh = size
    h, w = img.shape[:2]
    return _pass(_pass(img, pil_coeffs(w, ow), 1), pil_coeffs(h, oh), 0)


def pil_rotate_nearest(img, angle):
    """Image.rotate(angle, NEAREST, expand=False, fillcolor=0) of a uint8 [h, w, c] image."""
    angle = angle % 360.0
    if angle == 0:
        return img.copy()
    h, w = img.shape[:2]
    cx, cy = w / 2, h / 2
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0, round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    m[2] = m[0] * -cx + m[1] * -cy + m[2] + cx
    m[5] = m[3] * -cx + m[4] * -cy + m[5] + cy
    fix = lambda v: math.floor(v * 65536.0 + 0.5)  # noqa: E731
    a0, a1, a3, a4 = fix(m[0]), fix(m[1]), fix(m[3]), fix(m[4])
    a2, a5 = fix(m[2] + m[1] * 0.5 + m[0] * 0.5), fix(m[5] + m[4] * 0.5 + m[3] * 0.5)
    y, x = np.mgrid[0:h, 0:w].astype(np.int64)
    xin = (a2 + x * a0 + y * a1) >> 16
    yin = (a5 + x * a3 + y * a4) >> 16
    ok = (xin >= 0) & (xin < w) & (yin >= 0) & (yin < h)
    out = np.zeros_like(img)
    out[ok] = img[yin[ok], xin[ok]]
    return out


def pil_train_transform(img, flip, angle, size=224):
    """Resize((size, size)) -> RandomHorizontalFlip (flip bit 0) -> RandomVerticalFlip (bit 1) -> RandomRotation
    (angle) on a uint8 [h, w, 3] image, as uint8 (data_process.py:62-69 before ToTensor / Normalize)."""
    r = pil_resize_bilinear(img, (size, size))
    if flip & 1:
        r = r[:, ::-1]
    if flip & 2:
        r = r[::-1]
    return pil_rotate_nearest(np.ascontiguousarray(r), angle)
