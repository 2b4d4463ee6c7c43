"""CPU: the f2 media oracle (oracle/media.py) — STFT power against torch.stft, the Slaney filterbank's
defining properties, the cv2 fixed-point resize on exact cases, and the product's host-side constants
(deepfake_amd.media: DFT basis, filterbank) against the oracle's restatement.  librosa / cv2 are absent:
parity unpinned against them."""
import numpy as np
import torch

from oracle import media as OM


def test_stft_power_matches_torch_stft():
    g = np.random.default_rng(0)
    y = g.standard_normal(22050).astype(np.float32)
    p = OM.stft_power(y, 2048, 512)
    X = torch.stft(torch.from_numpy(y).double(), n_fft=2048, hop_length=512,
                   window=torch.hann_window(2048, periodic=True, dtype=torch.float64), center=True,
                   pad_mode="constant", return_complex=True)
    ref = (X.abs() ** 2).numpy()
    assert p.shape == ref.shape == (1025, 1 + 22050 // 512)
    assert np.abs(p - ref).max() <= 1e-9 * ref.max()


def test_slaney_filterbank_properties():
    fb = OM.mel_filters(22050, 2048, 128).astype(np.float64)
    assert fb.shape == (128, 1025) and (fb >= 0).all()
    freqs = np.linspace(0, 11025, 1025)
    # Slaney area normalisation: each triangle integrates (over Hz) to ~1 (up to the bin sampling)
    area = (fb * (freqs[1] - freqs[0])).sum(1)
    assert np.allclose(area[8:], 1.0, rtol=0.08)
    # band centres increase with the mel index; below 1 kHz the scale is linear (200/3 Hz per mel)
    peaks = freqs[fb.argmax(1)]
    assert (np.diff(peaks) >= 0).all()
    assert abs(OM.hz_to_mel(np.array([1000.0]))[0] - 15.0) < 1e-12
    assert abs(OM.mel_to_hz(OM.hz_to_mel(np.array([4321.0])))[0] - 4321.0) < 1e-9


def test_cv_resize_identity_and_constant():
    g = np.random.default_rng(1)
    img = g.integers(0, 256, size=(37, 53), dtype=np.uint8)
    assert np.array_equal(OM.cv_resize_linear_u8(img, (53, 37)), img)
    c = np.full((20, 30), 77, dtype=np.uint8)
    assert (OM.cv_resize_linear_u8(c, (224, 224)) == 77).all()


def test_product_constants_match_oracle():
    from deepfake_amd import media
    fb = media.mel_filterbank(22050, 2048, 128)
    assert np.allclose(fb, OM.mel_filters(22050, 2048, 128), rtol=1e-6, atol=1e-9)
    b = media.stft_basis(2048).astype(np.float64)
    g = np.random.default_rng(2)
    fr = g.standard_normal(2048)
    X = np.fft.rfft(fr * (0.5 - 0.5 * np.cos(2 * np.pi * np.arange(2048) / 2048)))
    got = fr @ b
    assert np.abs(got[:1025] - X.real).max() < 1e-4 and np.abs(got[1025:2050] - X.imag).max() < 1e-4
    assert b.shape == (2048, 2052) and not b[:, 2050:].any()


def _pil_cases():
    import golden_cases as GC
    from fixtures import load
    fx = load(GC.PIL_FRAMES["name"])
    shapes = {"resize720": (720, 1280, 3), "aug180": (180, 320, 3), "aug720": (720, 1280, 3), "mel224": (224, 224, 1),
              "aug_up": (100, 150, 3)}
    return GC, fx, shapes


def test_pil_restatement_matches_pil_fixtures():
    """oracle/media.py's PIL 12.2 restatement (antialiased BILINEAR resize, NEAREST rotation, flips) equals the
    fixtures PIL itself wrote (tests/golden/make_pil_fixtures.py), bit for bit."""
    GC, fx, shapes = _pil_cases()
    for name, (h, w, ch) in shapes.items():
        base = int(fx[name + ":seed"])
        for i in range(fx[name].shape[0]):
            img = GC.pil_test_image(base + i, h, w, ch)
            if ch == 1:
                img = np.repeat(img[..., None], 3, axis=2)
            if name == "resize720":
                got = OM.pil_resize_bilinear(img, (224, 224))
            else:
                got = OM.pil_train_transform(img, int(fx[name + ":flips"][i]), float(fx[name + ":angles"][i]))
            assert np.array_equal(got, fx[name][i]), (name, i, int((got != fx[name][i]).sum()))
    img = GC.pil_test_image(GC.PIL_FRAMES["seed"] * 1000 + 999, 720, 1280, 3)
    assert np.array_equal(OM.pil_resize_bilinear(img, (398, 224)), fx["eval720"][0])


def test_product_pil_constants_match_oracle():
    """The host-built constants the kernel reads (deepfake_amd.media: resize coefficients, rotation matrices)
    equal the oracle's restatement."""
    import math
    from deepfake_amd import media
    for n_in, n_out in ((1280, 224), (720, 224), (180, 224), (224, 224), (150, 224), (1280, 398)):
        b, k, ks = media.pil_bilinear_coeffs(n_in, n_out)
        taps = OM.pil_coeffs(n_in, n_out)
        for o, (x0, kv) in enumerate(taps):
            assert b[o, 0] == x0 and b[o, 1] == len(kv) and list(k[o, :len(kv)]) == kv and not k[o, len(kv):].any()
    for ang in (0.0, 37.5, -61.25, 90.0, 180.0, -89.99):
        m = media.pil_rotate_fixed(ang, 224, 224)
        assert (m[0] == 0) == (ang % 360.0 == 0)


def _scalar_draws(frames, generator, degrees=90.0):
    """The reference Compose's per-frame draw sequence (data_process.py:62-69): rand(1) < 0.5 twice, then
    RandomRotation's empty(1).uniform_(-90, 90), one frame after the other."""
    flips, angles = [], []
    for _ in range(frames):
        hf = bool(torch.rand(1, generator=generator) < 0.5)
        vf = bool(torch.rand(1, generator=generator) < 0.5)
        angles.append(float(torch.empty(1).uniform_(-degrees, degrees, generator=generator).item()))
        flips.append(int(hf) | (int(vf) << 1))
    return flips, angles


def test_draw_augment_matches_scalar_draws():
    """media.draw_augment's batched draw gives the per-frame scalar sequence bit for bit, and leaves the generator
    where the scalar loop leaves it."""
    from deepfake_amd import media
    for n in (1, 2, 17, 256):
        for seed in range(3):
            ga, gb = torch.Generator().manual_seed(seed), torch.Generator().manual_seed(seed)
            flips, angles = media.draw_augment(n, ga)
            rf, ra = _scalar_draws(n, gb)
            assert flips.dtype == torch.int32 and flips.tolist() == rf and angles == ra
            assert torch.equal(torch.rand(4, generator=ga), torch.rand(4, generator=gb))


def test_frame_augment_shape_contract():
    """RGB frames must be [..., H, W, 3]; grey images are routed by grey=True, never by a shape guess."""
    import pytest
    from deepfake_amd import media
    with pytest.raises(ValueError, match="RGB"):
        media.frame_augment(torch.zeros(2, 224, 224, dtype=torch.uint8))
    with pytest.raises(ValueError, match="RGB"):
        media.frame_augment(torch.zeros(224, 3, dtype=torch.uint8))
    with pytest.raises(ValueError, match="grey"):
        media.frame_augment(torch.zeros(5, dtype=torch.uint8), grey=True)
