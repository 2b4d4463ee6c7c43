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
  torchvision (tensor path): F.rotate (inverse affine grid of pixel centres, grid_sample nearest,
      fill 0), hflip / vflip, ToTensor, Normalize.
No golden vectors exist for these (the reference has no tests and the libraries are absent):
PARITY UNPINNED against librosa / cv2 / PIL; the STFT stage is checked against torch.stft.
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
