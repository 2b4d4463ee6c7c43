"""GPU: the f2 media front end (csrc/media.hip) against oracle/media.py and torch.
Mel image: the reference's generate_mel_spectrogram pipeline (src/utils.py:63-87) restated in numpy —
PARITY UNPINNED against librosa / cv2 (absent from the image); bars: at most 1 grey level apart, >= 99.5 %
of pixels identical (fp32 MFMA STFT vs float64 FFT: only values within ~1e-4 of a quantisation boundary flip).
Frame transform (data_process.py:62-69): flips bit-exact vs torch.flip, rotation vs torchvision's tensor
F.rotate restated with torch.nn.functional.grid_sample (nearest; >= 99.9 % identical, ties of the nearest
rounding may differ in the last fp32 ulp), resize vs torch F.interpolate(bilinear) rounded to uint8."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import media as OM

pytestmark = pytest.mark.gpu
DEV = "cuda"
MEAN = torch.tensor([0.485, 0.456, 0.406])
STD = torch.tensor([0.229, 0.224, 0.225])


def _norm(u8_chw):
    """T.ToTensor + T.Normalize on the CPU (IEEE division; torch's GPU division by a scalar multiplies by the
    reciprocal instead)."""
    x = u8_chw.cpu()
    return x.float().div(255).sub(MEAN.view(3, 1, 1)).div(STD.view(3, 1, 1))


@pytest.mark.parametrize("seconds", [1, 4])
def test_mel_image_matches_oracle(seconds):
    from deepfake_amd import media
    g = np.random.default_rng(seconds)
    S = 22050 * seconds
    t = np.arange(S) / 22050.0
    y = np.stack([0.3 * np.sin(2 * np.pi * 440 * t * (1 + 0.2 * t)) + 0.05 * g.standard_normal(S),
                  0.1 * g.standard_normal(S)]).astype(np.float32)
    got = media.mel_image(torch.from_numpy(y).to(DEV)).cpu().numpy()
    T = 1 + S // 512
    raw = media.mel_image(torch.from_numpy(y).to(DEV), size=(T, 128)).cpu().numpy()   # identity resize
    for b in range(2):
        ref_raw = OM.mel_db_uint8(y[b])
        d = np.abs(raw[b].astype(int) - ref_raw.astype(int))
        assert d.max() <= 1 and (d == 0).mean() >= 0.995, (d.max(), (d == 0).mean())
        ref = OM.cv_resize_linear_u8(ref_raw, (224, 224))
        d = np.abs(got[b].astype(int) - ref.astype(int))
        assert d.max() <= 1 and (d == 0).mean() >= 0.995, (d.max(), (d == 0).mean())
        # the resize itself is exact on the same uint8 input
        assert np.array_equal(OM.cv_resize_linear_u8(raw[b], (224, 224)), got[b])


def test_gray_normalize_exact():
    from deepfake_amd import media
    img = torch.randint(0, 256, (3, 224, 224), dtype=torch.uint8, device=DEV)
    out = media.gray_normalize(img).cpu()
    ref = torch.stack([_norm(i.unsqueeze(0).expand(3, -1, -1)) for i in img])
    assert torch.equal(out, ref)


def _rotate_ref(img_chw, angle):
    """torchvision.transforms.functional.rotate (tensor path, nearest, fill 0, expand False) restated."""
    C, h, w = img_chw.shape
    rot = math.radians(-angle)
    theta = torch.tensor([[math.cos(rot), math.sin(rot), 0.0], [-math.sin(rot), math.cos(rot), 0.0]],
                         dtype=torch.float32).view(1, 2, 3)
    base = torch.empty(1, h, w, 3)
    base[..., 0].copy_(torch.linspace(-w * 0.5 + 0.5, w * 0.5 + 0.5 - 1, steps=w))
    base[..., 1].copy_(torch.linspace(-h * 0.5 + 0.5, h * 0.5 + 0.5 - 1, steps=h).unsqueeze(-1))
    base[..., 2].fill_(1)
    grid = base.view(1, h * w, 3).bmm(theta.transpose(1, 2) / torch.tensor([0.5 * w, 0.5 * h])).view(1, h, w, 2)
    return F.grid_sample(img_chw.unsqueeze(0).float(), grid, mode="nearest", padding_mode="zeros",
                         align_corners=False)[0]


def test_frame_augment_flips_rotation_resize():
    from deepfake_amd import media
    from deepfake_amd import kernels as K
    n, H, W = 6, 224, 224
    fr = torch.randint(0, 256, (n, H, W, 3), dtype=torch.uint8, device=DEV)
    # identity transform == ToTensor + Normalize (dfk_frame_normalize), bit for bit
    assert torch.equal(media.frame_augment(fr), K.frame_normalize(fr))
    flips = torch.tensor([0, 1, 2, 3, 1, 2], dtype=torch.int32, device=DEV)
    out = media.frame_augment(fr, flips=flips).cpu()
    for i in range(n):
        x = fr[i].permute(2, 0, 1)
        if flips[i] & 1:
            x = torch.flip(x, [2])
        if flips[i] & 2:
            x = torch.flip(x, [1])
        assert torch.equal(out[i], _norm(x)), i
    angles = torch.tensor([0.0, 37.5, -90.0, 90.0, 12.25, -61.0], device=DEV)
    out = media.frame_augment(fr, flips=flips, angles=angles).cpu()
    for i in range(n):
        x = fr[i].permute(2, 0, 1).cpu()
        if flips[i] & 1:
            x = torch.flip(x, [2])
        if flips[i] & 2:
            x = torch.flip(x, [1])
        ref = _norm(_rotate_ref(x, float(angles[i])).round().to(torch.uint8))
        same = (out[i] == ref).all(0).float().mean().item()
        assert same >= 0.999, (i, same)
    # resize from a decoded 180x320 frame: torch bilinear (half-pixel centres) rounded to uint8
    src = torch.randint(0, 256, (2, 180, 320, 3), dtype=torch.uint8, device=DEV)
    out = media.frame_augment(src).cpu()
    ref = F.interpolate(src.permute(0, 3, 1, 2).float().cpu(), size=(224, 224), mode="bilinear", align_corners=False)
    ref = torch.stack([_norm(r.round().clamp(0, 255).to(torch.uint8)) for r in ref])
    same = (out == ref).all(1).float().mean().item()
    assert same >= 0.999, same


def test_trainer_media_inputs():
    """The trainer's device input path (deepfake_amd.trainer.prepare_video / prepare_mel) on a synthetic fused
    batch: uint8 frames with the training augmentation, the mel slot from a raw 22.05 kHz waveform and from the
    cached uint8 grey image — shapes, finiteness, and the eval path equal to plain ToTensor + Normalize."""
    from deepfake_amd.trainer import prepare_mel, prepare_video
    from deepfake_amd import kernels as K
    from deepfake_amd import media
    g = torch.Generator().manual_seed(0)
    frames = torch.randint(0, 256, (2, 4, 112, 112, 3), generator=g, dtype=torch.uint8)
    v = prepare_video(frames, DEV, augment=True)
    assert v.shape == (2, 4, 3, 224, 224) and torch.isfinite(v).all()
    v0 = prepare_video(frames, DEV, augment=False)
    assert torch.equal(v0, K.frame_normalize(frames.to(DEV)))
    wave = 0.1 * torch.randn(2, 22050 * 2, generator=g)
    m = prepare_mel(wave, DEV)
    assert m.shape == (2, 3, 224, 224) and torch.isfinite(m).all()
    assert torch.equal(m, media.gray_normalize(media.mel_image(wave.to(DEV))))
    gray = torch.randint(0, 256, (2, 224, 224), generator=g, dtype=torch.uint8)
    assert torch.equal(prepare_mel(gray, DEV), media.gray_normalize(gray.to(DEV)))
