"""GPU: the f2 media front end (csrc/media.hip) against oracle/media.py and torch.
Mel image: the reference's generate_mel_spectrogram pipeline (src/utils.py:63-87) restated in numpy —
PARITY UNPINNED against librosa / cv2 (absent from the image); bars: at most 1 grey level apart, >= 99.5 %
of pixels identical (fp32 MFMA STFT vs float64 FFT: only values within ~1e-4 of a quantisation boundary flip).
Frame / mel-image transform (data_process.py:55-69,162 — torchvision transforms on PIL images): bit-exact
against fixtures written by PIL 12.2 itself (tests/golden/pil_frames.npz: antialiased BILINEAR resize from
1280x720 / 320x180 / 150x100 frames, flips, NEAREST rotation, the eval shorter-side resize, the grey mel image),
then ToTensor + Normalize in fp32."""

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


@pytest.mark.parametrize("seconds", [1, 4, 14])   # 14 s: a 603-frame image, > 64 KB of LDS
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


def _pil_fixture():
    import golden_cases as GC
    from fixtures import load
    return GC, load(GC.PIL_FRAMES["name"])


@pytest.mark.parametrize("name,h,w,ch", [("resize720", 720, 1280, 3), ("aug180", 180, 320, 3), ("aug720", 720, 1280, 3),
                                         ("mel224", 224, 224, 1), ("aug_up", 100, 150, 3)])
def test_frame_augment_matches_pil(name, h, w, ch):
    """dfk_frame_augment (PIL resize + flips + rotation + ToTensor + Normalize) against PIL's own output,
    bit for bit; grey images (the mel JPEG) take the 1-channel path."""
    from deepfake_amd import media
    GC, fx = _pil_fixture()
    base, n = int(fx[name + ":seed"]), fx[name].shape[0]
    src = torch.from_numpy(np.stack([GC.pil_test_image(base + i, h, w, ch) for i in range(n)])).to(DEV)
    aug = name != "resize720"
    flips = torch.from_numpy(fx[name + ":flips"]) if aug else None
    angles = [float(a) for a in fx[name + ":angles"]] if aug else None
    out = media.frame_augment(src, flips=flips, angles=angles, grey=ch == 1).cpu()
    ref = torch.stack([_norm(torch.from_numpy(fx[name][i]).permute(2, 0, 1)) for i in range(n)])
    assert torch.equal(out, ref), int((out != ref).any(1).sum())


def test_frame_eval_resize_matches_pil():
    """Eval T.Resize(224) of a 1280x720 frame (shorter side to 224 -> 224 x 398) via prepare_video."""
    from deepfake_amd.trainer import prepare_video
    GC, fx = _pil_fixture()
    src = torch.from_numpy(GC.pil_test_image(GC.PIL_FRAMES["seed"] * 1000 + 999, 720, 1280, 3))[None, None]
    out = prepare_video(src, DEV, augment=False).cpu()
    assert out.shape == (1, 1, 3, 224, 398)
    assert torch.equal(out[0, 0], _norm(torch.from_numpy(fx["eval720"][0]).permute(2, 0, 1)))


def test_frame_augment_identity_and_flips():
    from deepfake_amd import media
    from deepfake_amd import kernels as K
    n = 4
    fr = torch.randint(0, 256, (n, 224, 224, 3), dtype=torch.uint8, device=DEV)
    assert torch.equal(media.frame_augment(fr), K.frame_normalize(fr))   # 224 -> 224: PIL's copy
    flips = torch.tensor([0, 1, 2, 3], dtype=torch.int32)
    out = media.frame_augment(fr, flips=flips).cpu()
    for i in range(n):
        x = fr[i].permute(2, 0, 1)
        if flips[i] & 1:
            x = torch.flip(x, [2])
        if flips[i] & 2:
            x = torch.flip(x, [1])
        assert torch.equal(out[i], _norm(x)), i


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
    f224 = torch.randint(0, 256, (2, 4, 224, 224, 3), generator=g, dtype=torch.uint8)
    assert torch.equal(prepare_video(f224, DEV, augment=False), K.frame_normalize(f224.to(DEV)))
    # the mel slot under --augment: the grey image through the frames' training transform (data_process.py:162),
    # the same draws as the frame path's for the same generator state
    gray0 = torch.randint(0, 256, (2, 224, 224), generator=g, dtype=torch.uint8)
    ga, gb = torch.Generator().manual_seed(5), torch.Generator().manual_seed(5)
    ma = prepare_mel(gray0, DEV, augment=True, generator=ga)
    flips, angles = media.draw_augment(2, gb)
    assert torch.equal(ma, media.frame_augment(gray0.to(DEV), flips=flips, angles=angles, grey=True))
    assert not torch.equal(ma, media.gray_normalize(gray0.to(DEV)))
    wave = 0.1 * torch.randn(2, 22050 * 2, generator=g)
    m = prepare_mel(wave, DEV)
    assert m.shape == (2, 3, 224, 224) and torch.isfinite(m).all()
    assert torch.equal(m, media.gray_normalize(media.mel_image(wave.to(DEV))))
    gray = torch.randint(0, 256, (2, 224, 224), generator=g, dtype=torch.uint8)
    assert torch.equal(prepare_mel(gray, DEV), media.gray_normalize(gray.to(DEV)))
