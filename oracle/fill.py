"""Deterministic named-hash weight fill + seeded synthetic inputs.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): used by tests/, the golden
generator, __graft_entry__.smoke() and bench.py's cpu_baseline leg.

There are no real checkpoints for the reference (every file under
/root/reference/checkpoints is a git-LFS pointer), so every
parity fixture is produced with weights filled by *parameter name*: the value
of a tensor depends only on (seed, state_dict key, shape).  The reference
model and the MI355X build share state_dict keys, so filling
both by name gives bit-identical weights without committing any weight file.

Rules (SURVEY.md §8c "Golden vectors"):
  * 1-D ``*.weight`` (LayerNorm / GroupNorm / BatchNorm affine) -> 1 + U(-.1,.1)
    (never zero: SwinV2's _init_respostnorm zeroes them, Q14)
  * biases and other 1-D tensors                          -> U(-.1,.1)
  * BatchNorm running_mean / running_var                  -> U(-.1,.1) / 1+U(0,.2)
  * relative_position_bias_table                          -> U(-.5,.5)
  * SwinV2 logit_scale                                    -> log(10) + U(-.2,.2)
  * weight-norm g (``original0``)                         -> U(.5,1.5)
  * every other >=2-D weight                              -> U(+-1/sqrt(fan_in))
  * integer buffers and the derived SwinV2 relative_coords_table are kept.
"""
import math
import zlib

import numpy as np
import torch

_KEEP = ("relative_position_index", "relative_coords_table", "num_batches_tracked", "attn_mask")


def _rng(seed, name):
    key = zlib.crc32(f"{int(seed)}::{name}".encode())
    return np.random.Generator(np.random.Philox(key=key))


def fill_value(name, shape, seed=0):
    """Return a float32 numpy array for state_dict key ``name``."""
    r = _rng(seed, name)
    n = int(np.prod(shape)) if len(shape) else 1
    if "running_var" in name:
        v = 1.0 + r.uniform(0.0, 0.2, n)
    elif "running_mean" in name:
        v = r.uniform(-0.1, 0.1, n)
    elif "relative_position_bias_table" in name:
        v = r.uniform(-0.5, 0.5, n)
    elif "logit_scale" in name:
        v = math.log(10.0) + r.uniform(-0.2, 0.2, n)
    elif name.endswith("original0"):
        v = r.uniform(0.5, 1.5, n)
    elif name.endswith("weight") and len(shape) == 1:
        v = 1.0 + r.uniform(-0.1, 0.1, n)
    elif name.endswith("bias") or len(shape) <= 1:
        v = r.uniform(-0.1, 0.1, n)
    else:
        fan_in = n // shape[0]
        b = 1.0 / math.sqrt(max(fan_in, 1))
        v = r.uniform(-b, b, n)
    return v.astype(np.float32).reshape(shape)


@torch.no_grad()
def named_fill_(module, seed=0):
    """Overwrite every floating parameter/buffer of ``module`` in place."""
    sd = module.state_dict(keep_vars=True)
    for name, t in sd.items():
        if any(k in name for k in _KEEP) or not torch.is_floating_point(t):
            continue
        t.copy_(torch.from_numpy(fill_value(name, tuple(t.shape), seed)).to(t.device, t.dtype))
    return module


def named_state(names_shapes, seed=0):
    """dict name -> float32 torch tensor for (name, shape) pairs (oracle side)."""
    return {n: torch.from_numpy(fill_value(n, tuple(s), seed)) for n, s in names_shapes}


def synthetic_inputs(B, T, H, W, seconds, mel=224, seed=1234):
    """SURVEY.md §8d synthetic batch: video [B,T,3,H,W], mel [B,3,mel,mel],
    waveform [B,16000*s] normalised per row (zero mean, unit var, eps 1e-7,
    HF feature_extraction_wav2vec2.py:94-95), labels in {0,1}."""
    def g(s):
        return np.random.Generator(np.random.Philox(key=s))
    video = g(seed).standard_normal((B, T, 3, H, W), dtype=np.float32)
    wave = g(seed + 1).standard_normal((B, int(16000 * seconds)), dtype=np.float32)
    wave = (wave - wave.mean(1, keepdims=True)) / np.sqrt(wave.var(1, keepdims=True) + 1e-7)
    melimg = g(seed + 2).standard_normal((B, 3, mel, mel), dtype=np.float32)
    label = (g(seed + 3).uniform(size=B) < 0.5).astype(np.float32)
    return (torch.from_numpy(video), torch.from_numpy(melimg),
            torch.from_numpy(wave.astype(np.float32)), torch.from_numpy(label))


def randn(key, shape, scale=1.0):
    """Seeded standard-normal float32 tensor (Philox, key -> stream)."""
    g = np.random.Generator(np.random.Philox(key=int(key)))
    return torch.from_numpy((g.standard_normal(tuple(shape), dtype=np.float32) * scale).astype(np.float32))
