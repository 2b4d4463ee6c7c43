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

Gradient accumulation (src/trainer.py:280-297, accum_step micro-batches per
optimizer step, default 4 at config.py:31): the non-final micro-steps run
inside ``no_sync()`` — arrivals are ignored, nothing is launched, gradients
just accumulate in the flat buffer — and only the last micro-step's backward
launches the bucket all-reduces, each over the sum of every micro-step.
"""
import contextlib
import os

import torch
import torch.distributed as dist


def recorder_on():
    """The process-group flight recorder is on (its size must be set before the process group exists)."""
    return max(int(os.environ.get(k, "0") or 0) for k in ("TORCH_FR_BUFFER_SIZE", "TORCH_NCCL_TRACE_BUFFER_SIZE")) > 0


def _fr_dumps():
    """The flight-recorder dump functions of this torch build (the NCCL/RCCL recorder and the generic one used
    by gloo are separate).  Raises when neither exists: without them the watchdog cannot be observed idle, and
    a capture that starts while it still polls an eager collective aborts the process."""
    from torch._C import _distributed_c10d as c10d
    dumps = [getattr(c10d, n) for n in ("_dump_nccl_trace_json", "_dump_fr_trace_json") if hasattr(c10d, n)]
    if not dumps:
        raise RuntimeError("this torch build exposes no flight-recorder dump (_dump_nccl_trace_json / "
                           "_dump_fr_trace_json): the RCCL watchdog cannot be observed idle")
    return dumps


def fr_entries():
    import json
    return [e for dump in _fr_dumps() for e in json.loads(dump(includeCollectives=True, onlyActive=False))
            .get("entries") or []]


def fr_last_id():
    """Highest flight-recorder record id so far (-1: none); brackets the collectives of one capture attempt."""
    return max((int(e.get("record_id", -1)) for e in fr_entries()), default=-1)


def watchdog_idle(timeout=60.0, exclude=()):
    """Wait until the flight recorder lists every collective as retired: the ProcessGroupNCCL watchdog marks a
    work retired in the same critical section in which it drops the work from the list it polls, so after that
    it queries none of their events again.  exclude: (lo, hi] record-id ranges of collectives recorded during a
    failed capture attempt (captured, never run: the watchdog never retires them).  Raises on timeout, and when
    the torch build has no flight recorder to poll."""
    import time
    _fr_dumps()
    t0 = time.monotonic()
    polls = 0
    while True:
        ents = [e for e in fr_entries()
                if not any(lo < int(e.get("record_id", -1)) <= hi for lo, hi in exclude)]
        live = [e for e in ents if not e.get("retired", False)]
        polls += 1
        if os.environ.get("DFK_DEBUG_WATCHDOG") and (polls == 1 or not live):
            print(f"[watchdog_idle] poll {polls} t={time.monotonic() - t0:.4f}s entries={len(ents)} live={len(live)} "
                  f"{[(e.get('profiling_name'), e.get('state')) for e in live[:4]]}", flush=True)
        if not live:
            return
        if time.monotonic() - t0 > timeout:
            raise RuntimeError(f"RCCL watchdog still tracks {len(live)} collectives after {timeout} s")
        time.sleep(0.002)


class GradBucketer:
    def __init__(self, store, bucket_mb=64.0, group=None, comm_dtype=torch.float32):
        self.store = store
        self.group = group
        # comm_dtype bf16: each bucket is cast to a bf16 copy right before its all-reduce (half the xGMI bytes:
        # 425 MB instead of 850 MB per C2 step) and the sum is cast back, / world, in finish()
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
        # DFK_DDP_FORCE=1 (tests / probes only): reduce even at one rank, so a 1-GPU box exercises the RCCL
        # launches, including their capture into the step's HIP graph
        self.enabled = self.world > 1 or (dist.is_initialized() and os.environ.get("DFK_DDP_FORCE") == "1")
        self.overlap = True       # hooks launch bucket all-reduces during backward (eager steps)
        self.sync = True          # False inside no_sync(): accumulation micro-steps launch nothing
        self.hooks = []
        self.bn_buffers = []
        self.streams = []         # branch streams whose kernels write gradients (FusionModel.branch_streams)
        self.comm_stream = None
        self.comm_dtype = comm_dtype
        self.cbuf = None
        if self.enabled and comm_dtype != torch.float32:
            self.cbuf = torch.zeros(store.grad.numel(), dtype=comm_dtype, device=store.grad.device)
        self.last_works = []      # the previous eager step's bucket works (drained before a graph capture)
        self.fr_exclude = []      # flight-recorder id ranges of failed capture attempts (see watchdog_idle)
        if self.enabled:
            for i, p in enumerate(store.params):
                self.hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
            store.listeners.append(self._ready)    # direct-mode gradients (no AccumulateGrad)
        self.reset()

    def reset(self):
        for b, (_, _, idx) in enumerate(self.buckets):
            self.pending[b] = len(idx)
            self.works[b] = None

    @contextlib.contextmanager
    def no_sync(self):
        """torch DDP.no_sync semantics: backward passes inside only accumulate."""
        old = self.sync
        self.sync = False
        try:
            yield
        finally:
            self.sync = old

    def _ready(self, i):
        if not (self.overlap and self.sync):
            return
        b = self.bucket_of[i]
        self.pending[b] -= 1
        if self.pending[b] == 0 and self.works[b] is None:
            self._launch(b)

    def _make_hook(self, i):
        return lambda _p: self._ready(i)

    def _payload(self, s, e):
        """The tensor all-reduced for flat range [s, e): the gradient itself, or its bf16 copy."""
        if self.cbuf is None:
            return self.store.grad[s:e]
        c = self.cbuf[s:e]
        c.copy_(self.store.grad[s:e])
        return c

    def _unpack(self):
        """Sum back into the fp32 gradient buffer, averaged over ranks."""
        if self.cbuf is None:
            self.store.grad.div_(self.world)
        else:
            self.store.grad.copy_(self.cbuf).div_(self.world)

    def _launch(self, b):
        s, e, _ = self.buckets[b]
        if not self.streams or not self.store.grad.is_cuda:
            self.works[b] = dist.all_reduce(self._payload(s, e), group=self.group, async_op=True)
            return
        # a bucket may hold gradients written on several branch streams: issue the all-reduce from a
        # comm stream that waits for all of them (RCCL orders itself after the issuing stream)
        if self.comm_stream is None:
            self.comm_stream = torch.cuda.Stream()
        cs = self.comm_stream
        cs.wait_stream(torch.cuda.current_stream())
        for st in self.streams:
            cs.wait_stream(st)
        with torch.cuda.stream(cs):
            self.works[b] = dist.all_reduce(self._payload(s, e), group=self.group, async_op=True)

    def drain(self, works=(), timeout=60.0):
        """Deterministic drain before a HIP-graph capture.  The ProcessGroupNCCL watchdog thread queries the
        events of every eager collective until it has seen it complete, and HIP refuses that query once the
        RCCL stream has joined a capture (the watchdog then aborts the process).  So: wait for the given
        works, idle the device, then poll the flight recorder (TORCH_FR_BUFFER_SIZE > 0, set by
        bench.py / train.py before the process group exists) until the watchdog has retired every eager
        collective of this process (watchdog_idle)."""
        for w in works:
            w.wait()
        if self.store.grad.is_cuda:
            torch.cuda.synchronize()
        if self.watched():
            watchdog_idle(timeout, exclude=self.fr_exclude)

    def watched(self):
        """A capture here needs the watchdog drain (RCCL on the device, flight recorder on)."""
        return self.enabled and self.store.grad.is_cuda and recorder_on()

    def fold_args(self):
        """What FusedSGD.step needs to consume the un-averaged all-reduce result directly (fold=True below):
        the 1 / world scale and, with bf16 buckets, the bf16 copy RCCL summed."""
        if not self.enabled:
            return {}
        return {"grad_scale": 1.0 / self.world, "grad_bf16": self.cbuf}

    def finish(self, fold=False):
        """After the last micro-step's backward: flush buckets not yet launched (unused
        parameters), wait for every bucket, average over ranks, re-arm the counters.
        fold=True: leave the SUM where RCCL put it (fp32 buffer or bf16 copy) and return fold_args() for the
        optimizer, which scales it in its own pass — no separate div_ / cast-back pass over the gradient
        (850 MB fp32 at C2, read and written once more per step)."""
        if not self.enabled:
            return {}
        for b in range(len(self.buckets)):
            if self.works[b] is None:
                self._launch(b)
        for w in self.works:
            w.wait()
        self.last_works = list(self.works)
        if not fold:
            self._unpack()
        self.reset()
        return self.fold_args() if fold else {}

    def allreduce_all(self, fold=False):
        """Non-overlapped variant (used outside a captured graph); fold as in finish()."""
        if not self.enabled:
            return {}
        works = [dist.all_reduce(self._payload(s, e), group=self.group, async_op=True) for s, e, _ in self.buckets]
        for w in works:
            w.wait()
        self.last_works = works
        if not fold:
            self._unpack()
        return self.fold_args() if fold else {}

    def track_batchnorm(self, module):
        """Remember the BatchNorm running statistics that broadcast_bn() refreshes every step."""
        self.bn_buffers = []
        for m in module.modules():
            if isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and m.track_running_stats:
                self.bn_buffers += [m.running_mean, m.running_var]
        return self

    def broadcast_bn(self, src=0):
        """Per-step BN running statistics from rank 0 (§8e): the reference's DataParallel
        re-replicates GPU0's module (buffers included) at every forward, so only GPU0's
        statistics persist; every rank starts each step from rank 0's."""
        if not self.enabled:
            return
        for buf in self.bn_buffers:
            dist.broadcast(buf, src, group=self.group)

    def broadcast_buffers(self, module, src=0):
        """All floating buffers from rank 0 (identical replicas at start-up)."""
        if not self.enabled:
            return
        for buf in module.buffers():
            if torch.is_floating_point(buf):
                dist.broadcast(buf, src, group=self.group)
