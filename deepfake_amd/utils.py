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
        self.drop = nn.Dropout(drop)
        self.p = drop

    def forward(self, x, residual=None):
        if self.p > 0 and self.training:
            h = Fn.linear(x, self.fc1.weight, self.fc1.bias, act=1)
            h = self.drop(h)
            y = self.drop(Fn.linear(h, self.fc2.weight, self.fc2.bias))
            return y if residual is None else y + residual
        return Fn.mlp(x, self.fc1, self.fc2, residual=residual)


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
