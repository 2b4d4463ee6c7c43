"""Flat parameter / gradient storage for the data-parallel training step.

Every trainable fp32 parameter becomes a view into one flat fp32 buffer, its
``.grad`` a view into one flat fp32 gradient buffer (so autograd accumulates in
place and buckets of the flat buffer are all-reduced as-is, no copies), and —
in bf16 compute mode — a bf16 shadow view (``p._dfk_shadow``) that the GEMMs
read.  The fused SGD kernel updates the fp32 master and rewrites the shadow in
the same pass, so no separate cast kernel runs per step.
Parameters are laid out in *reverse* registration order, which is roughly the
order in which backward produces their gradients (buckets in
reverse registration order), and each is 16-B aligned.
"""
import torch

from . import kernels as K

_ALIGN = 8  # elements (bf16 shadow views stay 16-B aligned)


class ParamStore:
    def __init__(self, model, compute_dtype=torch.float32, device=None):
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.params.reverse()
        dev = device or self.params[0].device
        self.offsets = []
        n = 0
        for p in self.params:
            self.offsets.append(n)
            n += -(-p.numel() // _ALIGN) * _ALIGN
        self.numel = n
        self.flat = torch.zeros(n, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(n, device=dev, dtype=torch.float32)
        self.shadow = torch.zeros(n, device=dev, dtype=torch.bfloat16) if compute_dtype == torch.bfloat16 else None
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                v = self.flat[o:o + p.numel()].view_as(p)
                v.copy_(p.data)
                p.data = v
                p.grad = self.grad[o:o + p.numel()].view_as(p)
                if self.shadow is not None:
                    p._dfk_shadow = self.shadow[o:o + p.numel()].view_as(p)
        self.refresh_shadow()

    def refresh_shadow(self):
        if self.shadow is not None:
            K.L.check(K.L.lib().dfk_cast(K.L.ptr(self.flat), K.L.F32, K.L.ptr(self.shadow), K.L.BF16, self.numel,
                                         K.L.stream()), "cast")

    def zero_grad(self):
        self.grad.zero_()

    def rebind_grads(self):
        """Re-attach .grad views (a user may have set grads to None)."""
        for p, o in zip(self.params, self.offsets):
            g = self.grad[o:o + p.numel()].view_as(p)
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g

    def span(self, i):
        p, o = self.params[i], self.offsets[i]
        return o, o + p.numel()
