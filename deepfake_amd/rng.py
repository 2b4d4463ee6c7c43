"""Device-side randomness of the training-mode regularisers (dropout, DropPath,
attention dropout, LayerDrop, SpecAugment).

The reference draws them from torch's generators (nn.Dropout, timm DropPath,
``torch.rand([])`` for LayerDrop, numpy for SpecAugment — HF
modeling_wav2vec2.py:101-218,700-706).  Here every mask is a counter-based hash
of (seed, step, site, row, col) evaluated inside the kernel that applies it
(include/dfk.h ``dfk_drop``): the seed and the step counter live in one device
tensor, the step is advanced by a device op once per training micro-step, so a
captured HIP graph draws new masks at every replay and the backward kernels
regenerate exactly the forward's mask without storing it.

State: int64[4] = [per-rank seed, step, shared seed, 0].  The shared seed is the
same on every data-parallel rank (LayerDrop coins must agree across replicas, or
the SGD skip of a dropped layer would diverge); the per-rank seed differs so the
element masks of different clip shards are independent.

Sites: every dropout site gets a distinct id at module construction
(``new_site``), in construction order, so identically built replicas agree.
"""
import itertools

import torch

_states = {}
_sites = itertools.count(1)
_seed = [0x5eed, 0xd15c0]   # per-rank base, shared


def new_site():
    return next(_sites)


def manual_seed(seed, rank=0):
    """Seed every device state: per-rank stream = f(seed, rank), shared stream = f(seed)."""
    _seed[0] = (int(seed) * 1000003 + int(rank) * 7919 + 0x5eed) & 0x7fffffffffffffff
    _seed[1] = (int(seed) * 2654435761 + 0xd15c0) & 0x7fffffffffffffff
    for st in _states.values():
        st[0], st[2] = _seed[0], _seed[1]
        st[1] = 0


def state(device):
    """The int64[4] device tensor the kernels read (created on first use)."""
    key = torch.device(device)
    if key.type == "cuda" and key.index is None:
        key = torch.device("cuda", torch.cuda.current_device())
    st = _states.get(key)
    if st is None:
        st = torch.tensor([_seed[0], 0, _seed[1], 0], dtype=torch.int64, device=key)
        _states[key] = st
    return st


def advance(device):
    """Next micro-step's masks (a device op: replays of a captured graph advance too)."""
    state(device)[1:2].add_(1)


class Drop:
    """One dropout site: mode 1 = element dropout, 2 = DropPath (one draw per `group_rows` rows).
    ``spec(rows_per_group)`` is what the kernel wrappers take (None when inactive)."""

    def __init__(self, p, mode=1, shared=False):
        self.p, self.mode, self.shared = float(p), int(mode), bool(shared)
        self.site = new_site()

    def active(self, training):
        return training and self.p > 0.0

    def spec(self, group_rows=1):
        return (self.mode, self.site, self.p, int(group_rows), int(self.shared))
