"""The entry surface of the reference on CPU: train.py / test.py flags (config.py), the cosine learning-rate
schedule, the synthetic DeepFakeSet / collate functions and the processor's padding.  CPU only."""
import json
import math
import os

import numpy as np
import pytest
import torch

from config import get_opt
from deepfake_amd.data import DeepFakeSet, IMAGENET_MEAN, IMAGENET_STD
from deepfake_amd.optim import CosineAnnealingLR
from deepfake_amd.trainer import pad_longest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_config_has_every_reference_flag():
    """All 31 flags of the reference's config.py:3-45 (tests/golden/config_flags.json, captured from the
    reference's own parser): same option strings, type and default."""
    ref = json.load(open(os.path.join(GOLD, "config_flags.json")))
    assert len(ref) == 31
    ours = get_opt([])
    from config import build_parser
    acts = {a.dest: a for a in build_parser()._actions}
    for f in ref:
        a = acts[f["dest"]]
        assert list(a.option_strings) == f["options"], f
        assert type(a).__name__ == f["action"], f
        assert getattr(a.type, "__name__", None) == f["type"], f
        assert getattr(ours, f["dest"]) == f["default"], f


def test_config_parses_reference_command_line():
    a = get_opt(["--modality", "fused", "-b", "8", "--accum_step", "4", "-lr", "1e-4", "-e", "2", "--l2_decacy", "0.05",
                 "--log_step", "5", "--Resume", "--fused_ckpt_path", "x.pth", "--config", "c1", "--dtype", "fp32"])
    assert (a.modality, a.batch_size, a.accum_step, a.epochs, a.Resume, a.config, a.dtype) == \
        ("fused", 8, 4, 2, True, "c1", "fp32")


class _Opt:
    def __init__(self, lr):
        self.base_lr = lr
        self.param_groups = [{"lr": lr}]

    def set_lr(self, lr):
        self.param_groups[0]["lr"] = lr


@pytest.mark.parametrize("T_max", [1, 7, 50])
def test_cosine_schedule_matches_torch(T_max):
    """src/trainer.py:85: torch.optim.lr_scheduler.CosineAnnealingLR(T_max), stepped once per optimizer step
    (also past T_max, where torch's recursive form keeps cycling)."""
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1e-4, momentum=0.9)
    ref = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=T_max)
    ours = CosineAnnealingLR(_Opt(1e-4), T_max=T_max)
    for _ in range(3 * T_max + 2):
        opt.step()
        ref.step()
        ours.step()
        r, o = opt.param_groups[0]["lr"], ours.opt.param_groups[0]["lr"]
        assert math.isclose(r, o, rel_tol=1e-6, abs_tol=1e-12), (r, o)


class _Args:
    batch_size, num_workers, modality, random_seed = 2, 0, "fused", 3
    train_clips, val_clips, test_clips, num_frames = 5, 3, 3, 4


@pytest.mark.parametrize("frames", ["normalized", "uint8"])
def test_synthetic_dataset_batches(frames):
    a = _Args()
    a.frames = frames
    ds = DeepFakeSet(a, clip_shape=dict(T=4, H=16, W=16, seconds=0.25))
    ds.setup()
    feat, label, names = next(iter(ds.train_dataloader()))
    assert set(feat) == {"Video", "Audio", "PAudio"} and len(names) == 2
    if frames == "uint8":
        assert feat["Video"].dtype == torch.uint8 and feat["Video"].shape == (2, 4, 16, 16, 3)
    else:
        assert feat["Video"].shape == (2, 4, 3, 16, 16) and feat["Video"].dtype == torch.float32
    assert feat["Audio"].shape == (2, 3, 224, 224)
    assert isinstance(feat["PAudio"], list) and feat["PAudio"][0].shape == (4000,)
    assert set(label.tolist()) <= {0.0, 1.0}
    assert len(ds.train_dataloader()) == 2                       # drop_last on the shuffled train split
    tf, tn = next(iter(ds.test_dataloader()))
    assert tn[0].startswith("synthetic_test_")
    # the same clip index is the same clip (seeded), uint8 normalised == the fp32 transform output
    a2 = _Args()
    a2.frames = "uint8" if frames == "normalized" else "normalized"
    other = DeepFakeSet(a2, clip_shape=dict(T=4, H=16, W=16, seconds=0.25))
    other.setup()
    u8 = (ds if frames == "uint8" else other).valset[1][0]["Video"]
    f32 = (other if frames == "uint8" else ds).valset[1][0]["Video"]
    ref = (u8.permute(0, 3, 1, 2).float() / 255 - torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)) \
        / torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
    assert torch.equal(ref, f32)


def test_processor_padding_longest():
    """padding='longest' (src/trainer.py:258): zeros after each shorter waveform (normalised afterwards
    over the whole padded row, Q13)."""
    w = pad_longest([np.ones(3, np.float32), np.arange(5, dtype=np.float32)])
    assert w.shape == (2, 5) and w[0].tolist() == [1, 1, 1, 0, 0] and w[1].tolist() == [0, 1, 2, 3, 4]


def test_check_finite_stops_on_nan_loss():
    """Failure detection at log steps: a NaN / Inf loss raises instead of being logged and stepped on."""
    import math
    import pytest
    from deepfake_amd.trainer import check_finite
    assert check_finite(0.69, 1) == 0.69
    for bad in (math.nan, math.inf, -math.inf):
        with pytest.raises(FloatingPointError):
            check_finite(bad, 3)
