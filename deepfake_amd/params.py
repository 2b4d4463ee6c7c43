"""Flat parameter / gradient storage for the data-parallel training step.

Every trainable fp32 parameter becomes a view into one flat fp32 buffer, its
``.grad`` a view into one flat fp32 gradient buffer (so autograd accumulates in
place and buckets of the flat buffer are all-reduced as-is, no copies), and —
in bf16 compute mode — a bf16 shadow view (``p._dfk_shadow``) that the GEMMs
read.  The fused SGD kernel updates the fp32 master and rewrites the shadow in
the same pass, so no separate cast kernel runs per step.

Direct mode (default): the HIP backward kernels accumulate weight gradients
straight into ``p.grad`` with fp32 atomics (deepfake_amd.functional.grad_sink)
and report the parameter ready through ``grad_ready`` — autograd then runs no
per-parameter zero-fill or AccumulateGrad add (~1600 small kernels per C2 step).
Parameters reached only through torch ops keep the AccumulateGrad path.
Parameters are laid out in *reverse* registration order, which is roughly the
order in which backward produces their gradients (buckets in
reverse registration order), and each is 16-B aligned.  Modules may ask for
adjacency groups (``flat_groups()``): parameters placed back to back in a given
order, optionally with zero gaps, so one GEMM reads them as a single operand —
wav2vec2's q/k/v projections as one [3C, C] weight and [3C] bias, SwinV2's
(q_bias, 0, v_bias) as the qkv bias — with no per-step concatenation, cast or
gradient scatter (``group_span``).  Gap elements are never stepped by the SGD.
"""
import torch

from . import kernels as K

_ALIGN = 8  # elements (bf16 shadow views stay 16-B aligned)
PARAM_BY_PTR = {}   # flat-buffer address -> parameter (resolves aliases handed back by checkpoint recomputes)


class ParamStore:
    def __init__(self, model, compute_dtype=torch.float32, device=None, direct=True):
        order = [p for p in model.parameters() if p.requires_grad]
        order.reverse()
        dev = device or order[0].device
        trainable = {id(p) for p in order}
        group_of = {}
        for m in model.modules():
            if hasattr(m, "flat_groups"):
                for grp in m.flat_groups():
                    ps = [e for e in grp if not isinstance(e, int)]
                    sizes = [e if isinstance(e, int) else e.numel() for e in grp]
                    if all(id(q) in trainable and id(q) not in group_of for q in ps) and \
                            all(z % _ALIGN == 0 for z in sizes):
                        for q in ps:
                            group_of[id(q)] = grp
        self.params, self.offsets = [], []
        placed = set()
        n = 0
        for p in order:
            grp = group_of.get(id(p))
            if grp is None:
                self.params.append(p)
                self.offsets.append(n)
                n += -(-p.numel() // _ALIGN) * _ALIGN
            elif id(grp[0] if not isinstance(grp[0], int) else grp[1]) not in placed:
                for e in grp:                 # the whole group back to back, in its own order
                    if isinstance(e, int):
                        n += e                # zero gap
                        continue
                    placed.add(id(e))
                    self.params.append(e)
                    self.offsets.append(n)
                    n += e.numel()
                placed.add(id(grp[0] if not isinstance(grp[0], int) else grp[1]))
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
                if direct:
                    p._dfk_store = self
                    PARAM_BY_PTR[p.data_ptr()] = p
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.uses = {}           # id(p) -> forward uses whose backward has not run yet (direct mode)
        self.listeners = []      # callbacks(i) when parameter i's gradient is complete
        # parameters that received a gradient since the last zero_grad: torch's SGD skips a
        # parameter whose .grad is None (no weight decay, no momentum), e.g. Audio2D.classifier
        # with use_feat=True (Q10) or a LayerDrop-skipped layer; FusedSGD steps only these
        self.touched = [False] * len(self.params)
        for i, p in enumerate(self.params):
            p.register_post_accumulate_grad_hook(self._mark(i))
        # device skip flags (LayerDrop): gate[i] is a 1-element fp32 tensor, 0 = leave parameter i untouched
        self.gate = [None] * len(self.params)
        self.gate_owners = []    # modules whose gates restart with every accumulation window (reset_gates)
        for m in model.modules():
            if hasattr(m, "param_gates"):
                if hasattr(m, "reset_gates") and m.param_gates():
                    self.gate_owners.append(m)
                for ps, flag in m.param_gates():
                    for p in ps:
                        i = self.index.get(id(p))
                        if i is not None:
                            self.gate[i] = flag
        self.refresh_shadow()

    def _mark(self, i):
        def hook(_p):
            self.touched[i] = True
        return hook

    def grad_ready(self, p):
        """A direct-mode backward finished accumulating into p.grad."""
        k = id(p)
        i = self.index[k]
        self.touched[i] = True
        n = self.uses.get(k, 1) - 1
        if n > 0:
            self.uses[k] = n
            return
        self.uses.pop(k, None)
        for cb in self.listeners:
            cb(i)

    def touched_runs(self, also=None, every=False):
        """Contiguous [start, end) element ranges of the flat buffers covering the touched
        parameters (every=True: all parameters), split where ``also[i]`` changes and at group gaps."""
        runs = []
        for i, t in enumerate(self.touched):
            if not (t or every):
                continue
            s, e = self.offsets[i], self.offsets[i] + self.params[i].numel()
            key = also[i] if also is not None else None
            adjacent = runs and s == -(-runs[-1][1] // _ALIGN) * _ALIGN
            if runs and runs[-1][2] == key and runs[-1][3] == i - 1 and adjacent:
                runs[-1] = (runs[-1][0], e, key, i)
            else:
                runs.append((s, e, key, i))
        return [(s, e, k) for s, e, k, _ in runs]

    def refresh_shadow(self):
        if self.shadow is not None:
            K.L.check(K.L.lib().dfk_cast(K.L.ptr(self.flat), K.L.F32, K.L.ptr(self.shadow), K.L.BF16, self.numel,
                                         K.L.stream()), "cast")

    def zero_gates(self):
        """Device ops only (captured into the step graph with the gradient zeroing)."""
        for m in self.gate_owners:
            m.reset_gates()

    def zero_grad(self):
        self.grad.zero_()
        self.zero_gates()
        self.uses.clear()
        self.touched = [False] * len(self.params)

    def rebind_grads(self):
        """Re-attach .grad views (a user may have set grads to None)."""
        for p, o in zip(self.params, self.offsets):
            g = self.grad[o:o + p.numel()].view_as(p)
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g

    def group_span(self, entries):
        """(start, length) of an adjacency group laid out as given (parameters and int gaps), or None."""
        first = next(e for e in entries if not isinstance(e, int))
        i = self.index.get(id(first))
        if i is None:
            return None
        lead = 0
        for e in entries:
            if e is first:
                break
            lead += e if isinstance(e, int) else e.numel()
        start = self.offsets[i] - lead
        o = start
        for e in entries:
            if isinstance(e, int):
                o += e
                continue
            j = self.index.get(id(e))
            if j is None or self.offsets[j] != o:
                return None
            o += e.numel()
        return start, o - start

    def span(self, i):
        p, o = self.params[i], self.offsets[i]
        return o, o + p.numel()
