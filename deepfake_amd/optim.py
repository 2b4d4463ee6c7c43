"""Fused SGD + CosineAnnealingLR over a ParamStore (src/trainer.py:80-85,295-297).

torch.optim.SGD(lr, momentum=0.9, weight_decay=wd) semantics (dampening 0,
no nesterov; first step buf = g) in one HBM-bound kernel over the flat fp32
buffer, which also rewrites the bf16 compute shadow.  The learning rate lives
in device memory so a captured graph replays with the scheduler's current lr.
"""
import math
import os

import torch

from . import kernels as K


# DFK_SGD_RUNS=0: one dfk_sgd_step launch per run (A/B); default: every run in one dfk_sgd_step_runs launch
_RUNS = os.environ.get("DFK_SGD_RUNS", "1") != "0"


class FusedSGD:
    def __init__(self, store, lr, momentum=0.9, weight_decay=0.0):
        self.store = store
        self.base_lr = float(lr)
        self.momentum, self.weight_decay = float(momentum), float(weight_decay)
        self.buf = torch.zeros_like(store.flat)
        self.lr_dev = torch.full((1,), self.base_lr, device=store.flat.device, dtype=torch.float32)
        self.param_groups = [{"lr": self.base_lr, "initial_lr": self.base_lr}]
        self.first = True
        self.has_buf = [False] * len(store.params)   # torch: momentum buffer created at a param's first grad

    def set_lr(self, lr):
        self.param_groups[0]["lr"] = float(lr)
        self.lr_dev.fill_(float(lr))

    def step(self, first=None, grad_scale=1.0, grad_bf16=None):
        """One SGD step over the parameters that received a gradient (torch skips grad=None:
        no weight decay and no momentum for them): every contiguous run in one dfk_sgd_step_runs launch (one
        dfk_sgd_step per run beyond 64 runs, or with DFK_SGD_RUNS=0).
        grad_scale / grad_bf16: the data-parallel fold of GradBucketer.finish(fold=True) — the gradient is the
        all-reduced sum (in the fp32 buffer, or in the bf16 bucket copy) times 1 / world."""
        st = self.store
        gates = {id(g): g for g in st.gate if g is not None}
        gkey = [id(g) if g is not None else None for g in st.gate]
        if not any(st.touched):          # no bookkeeping (e.g. a captured replay): every parameter
            f0 = self.first if first is None else first
            runs = st.touched_runs(also=[(f0, k) for k in gkey], every=True)
        else:
            runs = st.touched_runs(also=[(not h, k) for h, k in zip(self.has_buf, gkey)])
            for i, t in enumerate(st.touched):
                if t:
                    self.has_buf[i] = True
        # a LayerDrop-gated run is skipped on the device when its layer was dropped this step
        if _RUNS and 0 < len(runs) <= K.SGD_MAX_RUNS:
            K.sgd_step_runs(st.flat, st.grad, self.buf, st.shadow, [(s, e, gates.get(k), f) for s, e, (f, k) in runs],
                            self.momentum, self.weight_decay, self.lr_dev, grad_scale=grad_scale,
                            grad_bf16=grad_bf16)
            self.first = False
            return
        for s, e, (f, k) in runs:
            K.sgd_step(st.flat[s:e], st.grad[s:e], self.buf[s:e], st.shadow[s:e] if st.shadow is not None else None,
                       0.0, self.momentum, self.weight_decay, bool(f), lr_dev=self.lr_dev, gate=gates.get(k),
                       grad_scale=grad_scale, grad_bf16=grad_bf16[s:e] if grad_bf16 is not None else None)
        self.first = False

    def zero_grad(self):
        self.store.zero_grad()

    def state_dict(self):
        return {"momentum_buffer": self.buf, "lr": self.param_groups[0]["lr"], "first": self.first}


class CosineAnnealingLR:
    """torch.optim.lr_scheduler.CosineAnnealingLR (eta_min 0) closed form, stepped per optimizer step."""

    def __init__(self, optimizer, T_max, eta_min=0.0):
        self.opt, self.T_max, self.eta_min = optimizer, max(int(T_max), 1), eta_min
        self.t = 0

    def get_lr(self):
        base = self.opt.base_lr
        return self.eta_min + (base - self.eta_min) * (1 + math.cos(math.pi * self.t / self.T_max)) / 2

    def step(self):
        self.t += 1
        self.opt.set_lr(self.get_lr())
