"""Helpers to compare tensors with (possibly compressed) golden fixtures."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def keys(fx, prefix):
    out = set()
    for k in fx:
        if k.startswith(prefix):
            out.add(k.split("@")[0])
    return sorted(out)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def error(fx, key, t):
    """max|a-b| / max|b| of tensor t against fixture key (full array, or the @sub sample and the
    @norm of a compressed one, whichever is worse); raises on a shape mismatch only."""
    a = t.detach().float().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)
    if key in fx:
        assert a.shape == fx[key].shape, f"{key}: shape {a.shape} vs {fx[key].shape}"
        return rel_err(a, fx[key])
    step = int(fx[key + "@step"])
    assert tuple(a.shape) == tuple(fx[key + "@shape"]), f"{key}: shape"
    e = rel_err(a.reshape(-1)[::step], fx[key + "@sub"])
    nrm = float(np.sqrt((a.astype(np.float64) ** 2).sum()))
    return max(e, abs(nrm - float(fx[key + "@norm"])) / max(float(fx[key + "@norm"]), 1e-12))


def check(fx, key, t, rtol, what=""):
    """Compare tensor t to fixture key (full array, or @sub/@sum/@norm summary).
    Error is max|a-b| / max|b| (relative to the tensor's scale)."""
    a = t.detach().float().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)
    if key in fx:
        ref = fx[key]
        assert a.shape == ref.shape, f"{what}{key}: shape {a.shape} vs {ref.shape}"
        e = rel_err(a, ref)
        assert e <= rtol, f"{what}{key}: rel err {e:.3e} > {rtol}"
        return e
    step = int(fx[key + "@step"])
    assert tuple(a.shape) == tuple(fx[key + "@shape"]), f"{what}{key}: shape"
    sub = a.reshape(-1)[::step]
    e = rel_err(sub, fx[key + "@sub"])
    assert e <= rtol, f"{what}{key}@sub: rel err {e:.3e} > {rtol}"
    nrm = float(np.sqrt((a.astype(np.float64) ** 2).sum()))
    en = abs(nrm - float(fx[key + "@norm"])) / max(float(fx[key + "@norm"]), 1e-12)
    assert en <= rtol, f"{what}{key}@norm: rel err {en:.3e} > {rtol}"
    return e
