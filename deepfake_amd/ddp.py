"""Bucketed gradient all-reduce over RCCL (torch.distributed "nccl" backend on
ROCm), overlapped with backward — replaces the reference's single-process
torch.nn.DataParallel (src/trainer.py:74-75: per-step parameter broadcast from
GPU0 and rooted reduce-add of gradients).

One process per GPU.  Gradients live in the ParamStore's flat fp32 buffer
(reverse registration order ~ backward order), cut into ~bucket_mb buckets.
A post-accumulate-grad hook per parameter (or, for gradients the HIP kernels
write directly into the flat buffer, ParamStore.grad_ready) counts arrivals; when a bucket is
complete its slice is all-reduced asynchronously (RCCL runs on its own stream
and overlaps the rest of backward).  ``finish()`` waits for the buckets and
averages (sum / world, matching the mean BCE loss over the global batch).
Parameters that never receive a gradient (Audio2D.classifier with
use_feat=True, Q10) are handled by a final flush: every bucket not yet
launched is reduced in finish().  Works with the gloo backend for CPU tests.
"""
import torch
import torch.distributed as dist


class GradBucketer:
    def __init__(self, store, bucket_mb=64.0, group=None):
        self.store = store
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        cap = int(bucket_mb * (1 << 20) / 4)
        self.buckets = []           # (start, end, [param indices])
        cur, start, end = [], None, None
        for i in range(len(store.params)):
            s, e = store.span(i)
            if start is None:
                start = s
            cur.append(i)
            end = e
            if end - start >= cap:
                self.buckets.append((start, end, cur))
                cur, start = [], None
        if cur:
            self.buckets.append((start, end, cur))
        self.bucket_of = {}
        for b, (_, _, idx) in enumerate(self.buckets):
            for i in idx:
                self.bucket_of[i] = b
        self.pending = [0] * len(self.buckets)
        self.works = [None] * len(self.buckets)
        self.enabled = self.world > 1
        self.overlap = True       # hooks launch bucket all-reduces during backward (eager steps)
        self.hooks = []
        if self.enabled:
            for i, p in enumerate(store.params):
                self.hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
            store.listeners.append(self._ready)    # direct-mode gradients (no AccumulateGrad)
        self.reset()

    def reset(self):
        for b, (_, _, idx) in enumerate(self.buckets):
            self.pending[b] = len(idx)
            self.works[b] = None

    def _ready(self, i):
        if not self.overlap:
            return
        b = self.bucket_of[i]
        self.pending[b] -= 1
        if self.pending[b] == 0 and self.works[b] is None:
            self._launch(b)

    def _make_hook(self, i):
        return lambda _p: self._ready(i)

    def _launch(self, b):
        s, e, _ = self.buckets[b]
        self.works[b] = dist.all_reduce(self.store.grad[s:e], group=self.group, async_op=True)

    def finish(self):
        if not self.enabled:
            return
        for b in range(len(self.buckets)):
            if self.works[b] is None:
                self._launch(b)
        for w in self.works:
            w.wait()
        self.store.grad.div_(self.world)
        self.reset()

    def allreduce_all(self):
        """Non-overlapped variant (used outside a captured graph)."""
        if not self.enabled:
            return
        works = [dist.all_reduce(self.store.grad[s:e], group=self.group, async_op=True) for s, e, _ in self.buckets]
        for w in works:
            w.wait()
        self.store.grad.div_(self.world)

    def broadcast_buffers(self, module, src=0):
        """BatchNorm running stats from rank 0 (the reference's DP keeps GPU0's, §8e)."""
        if not self.enabled:
            return
        for buf in module.buffers():
            if torch.is_floating_point(buf):
                dist.broadcast(buf, src, group=self.group)
