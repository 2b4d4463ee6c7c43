"""The reference's training / inference entry surface on the GPU (src/trainer.py, src/submit.py, train.py,
test.py): one Trainer.train() optimizer step at C1 against the reference's own post-step parameters
(tests/golden/fused_c1.npz), a save_ckpt -> load_ckpt round trip in the reference's checkpoint format,
SubmitCtl's prediction.csv, and the on-device input normalisation (frames, waveform)."""
import types

import numpy as np
import pytest
import torch

import golden_cases as GC
from fixtures import keys, load
from oracle.fill import named_fill_, synthetic_inputs

pytestmark = pytest.mark.gpu
if torch.cuda.is_available():
    from deepfake_amd import kernels as K
    from deepfake_amd.models.fused import build_fused
    from deepfake_amd.submit import SubmitCtl
    from deepfake_amd.trainer import Trainer

DEV = "cuda"


def _args(**kw):
    a = dict(epochs=0, learning_rate=0.01, batch_size=2, modality="fused", model_save=0, log_step=1, accum_step=1,
             l2_decacy=0.05, dtype="fp32", bucket_mb=64.0, soft=0.01, classify_drop=0.0, swin_drop=0.0)
    a.update(kw)
    return types.SimpleNamespace(**a)


class _OneBatch:
    """A DeepFakeSet stand-in whose train split is the fused_c1 fixture's batch (src/utils.py fusion_collate
    layout: PAudio a list of waveforms)."""

    def __init__(self, c):
        video, mel, wave, label = synthetic_inputs(c["B"], c["T"], c["H"], c["W"], c["seconds"], seed=c["seed"] + 1)
        self.batch = ({"Video": video, "Audio": mel, "PAudio": [w.numpy() for w in wave]}, label,
                      [f"clip{i}" for i in range(c["B"])])

    def train_dataloader(self):
        return [self.batch]

    def val_dataloader(self):
        return None

    def test_dataloader(self):
        return [(self.batch[0], self.batch[2])]


def test_trainer_step_matches_reference():
    c = GC.FUSED_C1
    fx = load(c["name"])
    m = named_fill_(build_fused("c1", compute_dtype=torch.float32), c["seed"])
    tr = Trainer(m, _args(), torch.device(DEV), _OneBatch(c), compute_dtype=torch.float32)
    tr.train()
    torch.cuda.synchronize()
    names = dict(m.named_parameters())
    bad = []
    for k in keys(fx, "ps:"):
        ref = float(fx[k])
        got = float(names[k[3:]].detach().double().sum())
        if abs(got - ref) > 1e-4 * max(1.0, abs(ref)) + 1e-3:
            bad.append((k, got, ref))
    assert not bad, bad[:5]
    # CosineAnnealingLR stepped once: T_max = epochs(0)*steps -> max(.,1) = 1 -> lr = 0
    assert tr.optimizer.param_groups[0]["lr"] == pytest.approx(0.0, abs=1e-12)


def test_checkpoint_round_trip_and_submit(tmp_path):
    c = GC.FUSED_C1
    m = named_fill_(build_fused("c1", compute_dtype=torch.float32), c["seed"])
    tr = Trainer(m, _args(), torch.device(DEV), _OneBatch(c), compute_dtype=torch.float32)
    tr.train()
    path = str(tmp_path / "ck.pth")
    tr.save_ckpt(path, 0)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert set(ck) == {"epoch", "checkpoint", "optimizer"}
    m2 = named_fill_(build_fused("c1", compute_dtype=torch.float32), c["seed"] + 1)
    tr2 = Trainer(m2, _args(fused_ckpt_path=path), torch.device(DEV), _OneBatch(c), compute_dtype=torch.float32)
    tr2.load_ckpt(_args(fused_ckpt_path=path))
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a.cpu(), b.cpu()), k
    # inference on the loaded model: SubmitCtl -> prediction.csv (src/submit.py:79-120)
    sub = SubmitCtl(m2, _args(), torch.device(DEV), _OneBatch(c))
    out = tmp_path / "prediction.csv"
    res = sub.submit(str(out))
    rows = out.read_text().strip().splitlines()
    assert len(rows) == c["B"] and rows[0].startswith("clip0,")
    m.eval()
    with torch.no_grad():
        feat = tr._features(_OneBatch(c).batch[0])
        p = m(feat).float().cpu().numpy()
    assert np.allclose([res[f"clip{i}"] for i in range(c["B"])], p, rtol=1e-5, atol=1e-6)


def test_frame_normalize_bit_exact():
    g = torch.Generator().manual_seed(0)
    u8 = torch.randint(0, 256, (3, 5, 32, 48, 3), generator=g, dtype=torch.uint8)
    got = K.frame_normalize(u8.to(DEV)).cpu()
    mean = torch.tensor((0.485, 0.456, 0.406)).view(1, 1, 3, 1, 1)
    std = torch.tensor((0.229, 0.224, 0.225)).view(1, 1, 3, 1, 1)
    ref = u8.permute(0, 1, 4, 2, 3).float().div(255).sub(mean).div(std)      # T.ToTensor + T.Normalize
    assert torch.equal(got, ref)


def test_wave_normalize_matches_feature_extractor():
    """zero_mean_unit_var_norm (transformers feature_extraction_wav2vec2.py:94-95) of padded rows."""
    rng = np.random.default_rng(1)
    w = [rng.standard_normal(64000).astype(np.float32) * 0.3 + 0.05, rng.standard_normal(50000).astype(np.float32)]
    from deepfake_amd.trainer import pad_longest
    x = pad_longest(w)
    got = K.wave_normalize(x.to(DEV)).cpu().numpy()
    ref = np.stack([(r - r.mean()) / np.sqrt(r.var() + 1e-7) for r in x.numpy()])
    assert np.abs(got - ref).max() < 2e-5
