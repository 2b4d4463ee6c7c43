"""Shared module surface of /root/reference/src/utils.py that the hot path uses:
``Mlp`` (:242-260) plus the trainer's logging helpers (Logger :203-214,
AverageMeter :185-201, seed_torch :382-391) restated without the unused media
dependencies (cv2/librosa/GPUtil)."""
import os
import random
from datetime import datetime

import numpy as np
import torch
import torch.nn as nn

from . import functional as Fn
from . import rng


class Mlp(nn.Module):
    """src/utils.py:242-260 — fc1 -> GELU -> drop -> fc2 -> drop.  On the HIP
    path fc1+GELU+fc2 run as two MFMA GEMMs with fused bias/GELU epilogues."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)   # module tree / state_dict parity; the masks are the sites below
        self.p = drop
        # nn.Dropout is called twice per forward (after the GELU, after fc2): two independent draws, i.e. two
        # device dropout sites, fused into the fc1 and fc2 GEMM epilogues (created only when p > 0, so the site
        # numbering of dropout-free models is unchanged)
        self.sites = (rng.Drop(drop), rng.Drop(drop)) if drop > 0 else None

    def drop_specs(self):
        """(after-GELU, after-fc2) dropout specs, or (None, None) outside training / at p = 0."""
        if self.sites is None or not self.training:
            return None, None
        return self.sites[0].spec(), self.sites[1].spec()

    def forward(self, x, residual=None):
        da, do = self.drop_specs()
        return Fn.mlp(x, self.fc1, self.fc2, residual=residual, drop_act=da, drop_out=do)


class AverageMeter:
    """src/utils.py:185-201."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = self.avg = self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        if self.count > 0:
            self.avg = self.sum / self.count


class Logger:
    """src/utils.py:203-214 (timestamped lines appended to a file); log_dir None
    prints to stdout instead of crashing (Q15)."""

    def __init__(self, log_dir):
        self.log_dir = log_dir
        self.f = None
        if log_dir:
            os.makedirs(os.path.dirname(os.path.abspath(log_dir)), exist_ok=True)
            self.f = open(log_dir, "a")
            self.f.truncate(0)

    def __call__(self, string):
        print(datetime.now(), string, file=self.f, flush=True)


def seed_torch(seed):
    """src/utils.py:382-391 (cudnn flags are irrelevant: no MIOpen on this path, Q16)."""
    seed = int(seed)
    random.seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def _strip_module(sd, skip=None):
    """src/utils.py:269-289: drop the first 7 characters ('module.' of a DataParallel checkpoint) of every key."""
    return {k[7:]: v for k, v in sd.items() if not (skip and skip in k)}


def load_pre_fused(args, VE, AE, PAE, logger=print):
    """src/utils.py:262-292: fine-tuned single-modality checkpoints ({'checkpoint': state_dict} of a DataParallel
    model) into the fused model's extractors — audio (SwinV2) without its 'head' keys, strict=False; video and
    paudio strict.  torch.load(weights_only=True): tensors only."""
    for path, mod, skip, strict, what in ((getattr(args, "audio_ckpt_path", None), AE, "head", False, "Audio"),
                                          (getattr(args, "video_ckpt_path", None), VE, None, True, "Video"),
                                          (getattr(args, "paudio_ckpt_path", None), PAE, None, True, "PAudio")):
        if path is None:
            continue
        logger(f"==============> Loading weight {path} for {what} fine-tuning......")
        ck = torch.load(path, map_location="cpu", weights_only=True)["checkpoint"]
        mod.load_state_dict(_strip_module(ck, skip), strict=strict)
        logger(f"=> loaded successfully '{path}'")


def load_pretrained(config, model, logger=print):
    """src/utils.py:294-380 (the SwinV2 audio branch): {'checkpoint': state_dict} with relative_position_index /
    relative_coords_table / attn_mask dropped (re-initialised here), relative_position_bias_table and
    absolute_pos_embed bicubic-resized when their size differs, strict=False."""
    import torch.nn.functional as F
    path = config.audio_ckpt_path
    logger(f"==============> Loading weight {path} for fine-tuning......")
    state_dict = dict(torch.load(path, map_location="cpu", weights_only=True)["checkpoint"])
    for k in [k for k in state_dict if "relative_position_index" in k or "relative_coords_table" in k or
              "attn_mask" in k]:
        del state_dict[k]
    own = model.state_dict()
    for k in [k for k in state_dict if "relative_position_bias_table" in k]:
        t = state_dict[k]
        L1, nH1 = t.size()
        L2, nH2 = own[k].size()
        if nH1 != nH2:
            logger(f"Error in loading {k}, passing......")
        elif L1 != L2:
            S1, S2 = int(L1 ** 0.5), int(L2 ** 0.5)
            state_dict[k] = F.interpolate(t.permute(1, 0).view(1, nH1, S1, S1), size=(S2, S2),
                                          mode="bicubic").view(nH2, L2).permute(1, 0)
    for k in [k for k in state_dict if "absolute_pos_embed" in k]:
        t = state_dict[k]
        _, L1, C1 = t.size()
        _, L2, _ = own[k].size()
        if L1 != L2:
            S1, S2 = int(L1 ** 0.5), int(L2 ** 0.5)
            t = F.interpolate(t.reshape(-1, S1, S1, C1).permute(0, 3, 1, 2), size=(S2, S2), mode="bicubic")
            state_dict[k] = t.permute(0, 2, 3, 1).flatten(1, 2)
    msg = model.load_state_dict(state_dict, strict=False)
    logger(msg)
    logger(f"=> loaded successfully '{getattr(config, 'audio_pretrained_dir', path)}'")
