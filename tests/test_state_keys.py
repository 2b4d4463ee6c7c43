"""state_dict compatibility with the reference ("state-dict keys must be identical"):
the fused model's keys AND shapes — parameters and buffers (relative_position_index, attn_mask,
relative_coords_table, BatchNorm running statistics, the weight-norm parametrization) — equal the
reference's own fused model at C1 (371 keys) and C2 (899 keys), from tests/golden/state_keys.json
(written by tests/golden/make_golden.py importing /root/reference).  CPU only: construction only."""
import json
import os

import pytest
import torch

from deepfake_amd.models.fused import build_fused

REF = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "state_keys.json")))


@pytest.mark.parametrize("cfg,name", [("c1", "fused_c1"), ("c2", "fused_c2")])
def test_state_dict_keys_and_shapes(cfg, name):
    ref = [(k, tuple(s)) for k, s in REF[name]]
    got = [(k, tuple(v.shape)) for k, v in build_fused(cfg).state_dict().items()]
    assert len(got) == len(ref), (len(got), len(ref))
    missing = sorted(set(ref) - set(got))
    extra = sorted(set(got) - set(ref))
    assert not missing and not extra, (missing[:10], extra[:10])


def test_reference_checkpoint_loads_strict():
    """A state_dict shaped like the reference's (every key, every shape) loads with strict=True."""
    m = build_fused("c1")
    sd = {k: torch.zeros(s) for k, s in REF["fused_c1"]}
    for k, v in m.state_dict().items():       # integer buffers keep their dtype
        sd[k] = sd[k].to(v.dtype)
    m.load_state_dict(sd, strict=True)
