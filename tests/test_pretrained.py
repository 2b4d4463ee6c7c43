"""CPU: the pretrained-weight loaders against the reference's own loaders run on the same synthetic checkpoints
(tests/golden/pretrained.npz, make_golden.py case_pretrained importing /root/reference):
SwinTransformer3D.inflate_weights / init_weights (video_swin_transformer.py:566-666: 2-D -> 3-D patch-embed repeat
divided by the patch depth, bicubic relative-position-bias resize, repeat 2Wd-1, re-initialised index buffers) and
the SwinV2 load_pretrained (src/utils.py:294-380); load_pre_fused (src/utils.py:262-292) by its key handling.
Checkpoints load with torch.load(weights_only=True)."""
import os
import types

import pytest
import torch

import golden_cases as GC
from fixtures import check, keys, load

from deepfake_amd.models.swin_transformer2d import SwinTransformerV2
from deepfake_amd.models.video_swin_transformer import SwinTransformer3D
from deepfake_amd.utils import load_pre_fused, load_pretrained


def test_inflate_weights_matches_reference(tmp_path):
    c = GC.PRETRAINED
    fx = load(c["name"])
    m = SwinTransformer3D(**c["vst"])
    ck = GC.synth_swin2d_checkpoint({k: tuple(v.shape) for k, v in m.state_dict().items()}, c["seed"])
    path = str(tmp_path / "swin2d.pth")
    torch.save(ck, path)
    m.init_weights(path)          # pretrained2d: inflate
    sd = m.state_dict()
    ks = keys(fx, "v:")
    assert len(ks) > 100
    for k in ks:
        check(fx, k, sd[k[2:]], 1e-6, what="inflate ")
    # the re-initialised buffers are this model's own, not the checkpoint's zeros
    assert sd["layers.0.blocks.0.attn.relative_position_index"].max() > 0
    assert sd["patch_embed.proj.weight"].shape == (96, 3, 2, 4, 4)


def test_swinv2_load_pretrained_matches_reference(tmp_path):
    c = GC.PRETRAINED
    fx = load(c["name"])
    m = SwinTransformerV2(**c["mel"])
    ck = GC.synth_swinv2_checkpoint({k: tuple(v.shape) for k, v in m.state_dict().items()}, c["seed"] + 1)
    path = str(tmp_path / "swinv2.pth")
    torch.save(ck, path)
    load_pretrained(types.SimpleNamespace(audio_ckpt_path=path, audio_pretrained_dir=path), m, logger=lambda *a: None)
    sd = m.state_dict()
    for k in keys(fx, "a:"):
        check(fx, k, sd[k[2:]], 1e-6, what="swinv2 ")
    assert not torch.equal(sd["layers.0.blocks.0.attn.relative_coords_table"],
                           torch.full_like(sd["layers.0.blocks.0.attn.relative_coords_table"], 7.0))


def test_load_pre_fused_key_handling(tmp_path):
    """'module.' stripped from every key; the audio extractor skips 'head' keys and loads strict=False; video and
    paudio load strict (a missing key raises)."""
    a, v, p = torch.nn.Linear(4, 3), torch.nn.Linear(5, 2), torch.nn.Linear(6, 2)
    g = torch.Generator().manual_seed(0)

    def ck(mod, extra=None):
        sd = {"module." + k: torch.randn(t.shape, generator=g) for k, t in mod.state_dict().items()}
        sd.update(extra or {})
        return {"checkpoint": sd}
    cka = ck(a, {"module.head.weight": torch.ones(2, 2)})
    ckv, ckp = ck(v), ck(p)
    paths = {}
    for name, obj in (("a", cka), ("v", ckv), ("p", ckp)):
        paths[name] = str(tmp_path / f"{name}.pth")
        torch.save(obj, paths[name])
    args = types.SimpleNamespace(audio_ckpt_path=paths["a"], video_ckpt_path=paths["v"], paudio_ckpt_path=paths["p"])
    load_pre_fused(args, v, a, p, logger=lambda *x: None)
    assert torch.equal(a.weight, cka["checkpoint"]["module.weight"])
    assert torch.equal(v.bias, ckv["checkpoint"]["module.bias"])
    assert torch.equal(p.weight, ckp["checkpoint"]["module.weight"])
    bad = {"checkpoint": {"module.weight": torch.zeros(2, 5)}}    # bias missing: strict video load raises
    torch.save(bad, paths["v"])
    with pytest.raises(RuntimeError):
        load_pre_fused(types.SimpleNamespace(audio_ckpt_path=None, video_ckpt_path=paths["v"], paudio_ckpt_path=None),
                       v, a, p, logger=lambda *x: None)
