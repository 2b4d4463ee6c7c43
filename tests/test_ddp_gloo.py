"""CPU, world_size 2 (gloo): the flat-buffer gradient bucketer reproduces the
single-process gradient of the global batch (mean loss), both with the
overlapped hook path and the non-overlapped path, tolerates parameters that
never receive a gradient (Audio2D.classifier, Q10), and broadcasts buffers."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deepfake_amd import functional as Fn
from deepfake_amd.ddp import GradBucketer
from deepfake_amd.params import ParamStore


class _DirectLinear(torch.autograd.Function):
    """CPU stand-in for a HIP backward that accumulates straight into p.grad
    (the direct-gradient protocol of deepfake_amd.functional)."""

    @staticmethod
    def forward(ctx, x, w, b):
        Fn.grad_use(ctx, 1, w)
        Fn.grad_use(ctx, 2, b)
        ctx.save_for_backward(x, w, b)
        return x @ w.t() + b

    @staticmethod
    def backward(ctx, dy):
        x, w, b = ctx.saved_tensors
        dw = Fn.grad_sink(w)
        dw += dy.t() @ x
        db = Fn.grad_sink(b)
        db += dy.sum(0)
        return dy @ w, Fn.grad_done(w, dw), Fn.grad_done(b, db)


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(16, 32)
        self.b = torch.nn.Linear(32, 8)
        self.c = torch.nn.Linear(32, 32)
        self.unused = torch.nn.Linear(4, 4)         # never used: grad stays 0 (Q10)
        self.bn = torch.nn.BatchNorm1d(8)

    def forward(self, x):
        h = torch.relu(self.a(x))
        h = h + _DirectLinear.apply(h, self.c.weight, self.c.bias)   # direct-mode parameters, used once
        return self.bn(self.b(h)).sum(-1)


def _free_port():
    """A TCP port free right now on 127.0.0.1 (fixed ports collide with sockets of an earlier test in TIME_WAIT)."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _data(seed, n):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 16, generator=g), torch.randn(n, generator=g)


def _worker(rank, world, port, overlap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = Net()
    store = ParamStore(m, torch.float32, device=torch.device("cpu"))
    bk = GradBucketer(store, bucket_mb=0.0002)  # tiny buckets (~52 floats) -> several buckets
    assert len(bk.buckets) >= 2
    bk.overlap = overlap                        # non-overlapped: hooks off, one reduce pass after backward
    x, y = _data(1, 8)
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
    loss = ((m(xs) - ys) ** 2).mean()
    loss.backward()
    if overlap:
        bk.finish()
    else:
        bk.allreduce_all()
    if rank == 0:
        m.bn.running_mean.fill_(3.0)
    bk.broadcast_buffers(m)
    q.put((rank, store.grad.numpy().copy(), m.bn.running_mean.numpy().copy()))   # by value: the worker exits
    dist.destroy_process_group()


class ProbNet(Net):
    def forward(self, x):
        return torch.sigmoid(super().forward(x[0]))


class _PlainSGD:
    """CPU stand-in for FusedSGD (the HIP kernel): flat -= lr * grad."""

    def __init__(self, store, lr):
        self.store, self.lr = store, lr

    def step(self):
        self.store.flat.add_(self.store.grad, alpha=-self.lr)


def _label(seed, n):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(n, generator=g) < 0.5).float()


ACC, MB = 2, 2   # micro-steps per optimizer step, clips per micro-batch per rank


def _accum_worker(rank, world, port, q):
    from deepfake_amd.trainer import TrainStep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = ProbNet()
    m.train()
    store = ParamStore(m, torch.float32, device=torch.device("cpu"))
    bk = GradBucketer(store, bucket_mb=0.0002)
    step = TrainStep(m, store, _PlainSGD(store, 0.1), bk)
    x, _ = _data(2, world * ACC * MB)
    lab = _label(3, world * ACC * MB)
    launched_early = []
    if rank == 0:
        m.bn.running_mean.fill_(5.0)      # rank 0's statistics win at the next step's broadcast
    for k in range(ACC):
        i0 = (rank * ACC + k) * MB
        step.micro((x[i0:i0 + MB],), lab[i0:i0 + MB], last=(k == ACC - 1), accum=ACC)
        if k < ACC - 1:
            launched_early.append(any(w is not None for w in bk.works))
    step.bucketer.broadcast_bn()
    q.put((rank, store.flat.numpy().copy(), m.bn.running_mean.numpy().copy(), launched_early))
    dist.destroy_process_group()


def test_accumulation_no_sync_matches_single_process_sum():
    """world 2 x accum_step 2 == one process summing the 4 micro-batches (each loss / 4), then one SGD
    step; non-final micro-steps launch no all-reduce (no_sync); BN statistics follow rank 0."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_accum_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (torch.from_numpy(f), torch.from_numpy(rm), le)) for r, f, rm, le in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
    torch.manual_seed(0)
    m = ProbNet()
    m.train()
    store = ParamStore(m, torch.float32, device=torch.device("cpu"))
    x, _ = _data(2, 2 * ACC * MB)
    lab = _label(3, 2 * ACC * MB)
    for j in range(2 * ACC):
        p = m((x[j * MB:(j + 1) * MB],))
        (torch.nn.BCELoss()(p, lab[j * MB:(j + 1) * MB]) / (2 * ACC)).backward()
    store.flat.add_(store.grad, alpha=-0.1)
    for r in range(2):
        f, rm, le = res[r]
        assert not any(le), "an all-reduce was launched inside no_sync"
        assert torch.allclose(f, store.flat, atol=1e-6), (r, (f - store.flat).abs().max())
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("overlap", [True, False])
def test_bucketed_allreduce_matches_global_batch(overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, overlap, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (torch.from_numpy(g), torch.from_numpy(rm))) for r, g, rm in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
    # reference: per-shard BN statistics, gradient averaged over the 2 shards (= DDP semantics)
    torch.manual_seed(0)
    m = Net()
    store = ParamStore(m, torch.float32, device=torch.device("cpu"))
    x, y = _data(1, 8)
    for r in range(2):
        loss = ((m(x[r * 4:(r + 1) * 4]) - y[r * 4:(r + 1) * 4]) ** 2).mean() / 2
        loss.backward()
    ref = store.grad
    for r in range(2):
        assert torch.allclose(res[r][0], ref, atol=1e-6), (r, (res[r][0] - ref).abs().max())
        assert torch.all(res[r][1] == 3.0)


def _layout_worker(rank, world, port, comm, q):
    """The real fused C1 model's parameter list in the ParamStore (reverse registration order, adjacency groups,
    16-B aligned gaps, 4 MB buckets): CPU stand-in gradients reported ready in backward order through the
    direct-gradient protocol (ParamStore.grad_ready), as the HIP backward kernels report them."""
    from deepfake_amd.models.fused import build_fused
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = build_fused("c1")
    store = ParamStore(m, torch.float32, device=torch.device("cpu"))
    bk = GradBucketer(store, bucket_mb=4.0, comm_dtype=comm)
    launched = []
    for i in range(len(store.params)):
        p = store.params[i]
        g = torch.Generator().manual_seed(1000 * rank + i)
        p.grad.copy_(torch.randn(p.shape, generator=g))
        store.grad_ready(p)
        launched.append(sum(w is not None for w in bk.works))
    bk.finish()
    q.put((rank, store.grad.numpy().copy(), launched, len(bk.buckets)))
    dist.destroy_process_group()


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_fused_model_bucket_layout(comm):
    """world 2: the bucketed all-reduce over the real fused C1 parameter layout (341 tensors, 49.4 M values)
    gives the mean of the ranks' gradients; buckets launch during the backward, not all at the end.
    bf16 buckets (half the xGMI bytes): within 8e-3 of the fp32 mean relative to each element's scale
    (one bf16 rounding per rank's value and one per partial sum)."""
    from deepfake_amd.models.fused import build_fused
    dt = torch.bfloat16 if comm == "bf16" else torch.float32
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_layout_worker, args=(r, 2, port, dt, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (torch.from_numpy(g), la, nb)) for r, g, la, nb in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
    m = build_fused("c1")
    store = ParamStore(m, torch.float32, device=torch.device("cpu"))
    ref = torch.zeros_like(store.grad)
    scale = torch.zeros_like(store.grad)
    for rank in range(2):
        for i, p in enumerate(store.params):
            g = torch.Generator().manual_seed(1000 * rank + i)
            s, e = store.span(i)
            v = torch.randn(p.shape, generator=g).reshape(-1)
            ref[s:e] += v / 2
            scale[s:e] += v.abs() / 2
    for r in range(2):
        got, launched, nb = res[r]
        assert nb > 4 and launched[len(launched) // 2] > 0, "buckets must launch during the backward"
        if comm == "fp32":
            assert torch.allclose(got, ref, atol=1e-6, rtol=0)
        else:
            assert bool(((got - ref).abs() <= 8e-3 * scale + 1e-6).all()), float((got - ref).abs().max())
    assert torch.equal(res[0][0], res[1][0])


class _Args:
    epochs, learning_rate, batch_size, modality, model_save, log_step = 1, 0.1, 2, "fused", 0, 1
    accum_step, l2_decacy, random_seed, bucket_mb = 1, 0.0, 42, 1.0


class _Data:
    def train_dataloader(self):
        return []

    def val_dataloader(self):
        return None


def _seed_worker(rank, world, port, q):
    from deepfake_amd import rng
    from deepfake_amd.trainer import Trainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    Trainer(Net(), _Args(), torch.device("cpu"), _Data(), compute_dtype=torch.float32)
    q.put((rank, rng.state("cpu").tolist()))
    dist.destroy_process_group()


def test_trainer_seeds_device_rng_per_rank():
    """Trainer seeds the device regulariser streams from --random_seed and the rank: element masks differ
    per rank (independent clip shards), the LayerDrop stream is shared (identical skips on every replica)."""
    from deepfake_amd import rng
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seed_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    st = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert st[0][0] != st[1][0]
    assert st[0][2] == st[1][2]
    rng.manual_seed(42, 1)
    assert rng.state("cpu").tolist()[0] == st[1][0]


def _agree_worker(rank, world, port, fail, q):
    """TrainStep._graph on CPU with the capture mechanics stubbed: `fail` names what breaks on rank 1 at the
    first form ('capture': the capture body raises; 'drain': the pre-capture watchdog drain times out).  Every
    rank must still reach _agree's MIN all-reduce and all must commit to the same (second) form."""
    from deepfake_amd.trainer import TrainStep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCH_FR_BUFFER_SIZE="2000")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = ProbNet()
    store = ParamStore(m, torch.float32, device=torch.device("cpu"))
    bk = GradBucketer(store, bucket_mb=0.0002)
    step = TrainStep(m, store, _PlainSGD(store, 0.1), bk)
    calls = []

    def capture_once(body, overlap, bn):
        calls.append((overlap, bn))
        if fail == "capture" and rank == 1 and len(calls) == 1:
            raise RuntimeError("stub: this form cannot be captured here")
        return "graph", ("outs", overlap, bn)

    real_drain = bk.drain
    drains = []

    def drain(works=(), timeout=60.0):
        drains.append(1)
        if fail == "drain" and rank == 1 and len(drains) == 1:
            raise RuntimeError("stub: RCCL watchdog still tracks 1 collectives")
        return real_drain(works, timeout)

    step._capture_once = capture_once
    bk.drain = drain
    g, outs, form = step._graph(lambda o, b: None, TrainStep.FORMS)
    q.put((rank, g, form, len(calls), bk.overlap))
    dist.destroy_process_group()


@pytest.mark.parametrize("fail", ["capture", "drain"])
def test_capture_failure_on_one_rank_moves_all_ranks(fail):
    """A rank whose capture (or pre-capture drain) fails alone does not diverge: all ranks drop the overlapped
    form together and commit to the one-pass form (src/trainer.py:74-75 replaced by per-GPU DDP, §8e)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, fail, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, form, n, ov)) for r, g, form, n, ov in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        g, form, n, ov = res[r]
        assert g == "graph" and form == (False, True), (r, res[r])
        assert ov is True      # the bucketer is left in its eager (hooked) state
    assert res[0][2] == 2 and res[1][2] == (2 if fail == "capture" else 1)


@pytest.mark.parametrize("world", [4])
def test_bf16_buckets_world4(world):
    """world 4, bf16 buckets over the real fused C1 layout: every rank's value is rounded to bf16 once and the
    ring sums up to world-1 partials in bf16, so |got - mean| <= (2*world-1) * 2^-9 * mean(|v|) per element
    (each rounding is at most 2^-9 of the magnitude it rounds)."""
    from deepfake_amd.models.fused import build_fused
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_layout_worker, args=(r, world, port, torch.bfloat16, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, g) for r, g, _, _ in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
    m = build_fused("c1")
    store = ParamStore(m, torch.float32, device=torch.device("cpu"))
    ref = torch.zeros_like(store.grad)
    scale = torch.zeros_like(store.grad)
    for rank in range(world):
        for i, p in enumerate(store.params):
            g = torch.Generator().manual_seed(1000 * rank + i)
            s, e = store.span(i)
            v = torch.randn(p.shape, generator=g).reshape(-1)
            ref[s:e] += v / world
            scale[s:e] += v.abs() / world
    bound = (2 * world - 1) * 2.0 ** -9
    for r in range(world):
        got = torch.from_numpy(res[r])
        assert bool(((got - ref).abs() <= bound * scale + 1e-6).all()), float(((got - ref).abs() / (scale + 1e-6)).max())
        assert torch.equal(got, torch.from_numpy(res[0]))


def test_watchdog_idle_raises_without_flight_recorder(monkeypatch):
    """No flight-recorder dump in this torch build: the drain must raise, not return at once (an empty entry
    list would otherwise read as 'watchdog idle' and the capture abort race would come back silently)."""
    from torch._C import _distributed_c10d as c10d
    from deepfake_amd import ddp
    for n in ("_dump_nccl_trace_json", "_dump_fr_trace_json"):
        monkeypatch.delattr(c10d, n, raising=False)
    with pytest.raises(RuntimeError, match="flight-recorder"):
        ddp.watchdog_idle(timeout=0.1)


def _finite_worker(rank, world, port, q):
    from deepfake_amd.trainer import check_finite
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = []
    for step, losses in ((1, (0.7, 0.69)), (2, (0.6, float("nan"))), (3, (float("inf"), 0.5))):
        try:
            check_finite(losses[rank], step, dist.group.WORLD)
            res.append("ok")
        except FloatingPointError as e:
            res.append("raise:" + ("other" if "another rank" in str(e) else "own"))
    q.put((rank, res))
    dist.destroy_process_group()


def test_check_finite_raises_on_every_rank():
    """A non-finite loss on one rank makes EVERY rank raise at that log step (the flag is MAX-all-reduced), so the
    healthy ranks do not block in the next gradient all-reduce until the RCCL watchdog fires."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_finite_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == ["ok", "raise:other", "raise:own"], res
    assert res[1] == ["ok", "raise:own", "raise:other"], res


def _fold_worker(rank, world, port, comm, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = Net()
    store = ParamStore(m, torch.float32, device=torch.device("cpu"))
    bk = GradBucketer(store, bucket_mb=0.0002, comm_dtype=comm)
    x, y = _data(1, 8)
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
    ((m(xs) - ys) ** 2).mean().backward()
    local = store.grad.clone()
    fa = bk.finish(fold=True)
    src = fa["grad_bf16"].float() if fa["grad_bf16"] is not None else store.grad
    q.put((rank, local.numpy().copy(), src.numpy().copy(), fa["grad_scale"],
           store.grad.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("comm", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_finish_fold_leaves_sum_and_scale(comm):
    """finish(fold=True): no averaging pass — the all-reduced SUM stays where RCCL put it (the fp32 gradient
    buffer, or the bf16 bucket copy while the fp32 buffer keeps the rank-local gradient) and the optimizer gets
    grad_scale = 1 / world (FusedSGD folds both into its one pass over the parameters)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fold_worker, args=(r, 2, port, comm, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
    total = torch.from_numpy(res[0][0]) + torch.from_numpy(res[1][0])
    for r in range(2):
        local, src, scale, gbuf = (torch.from_numpy(v) if not isinstance(v, float) else v for v in res[r])
        assert scale == 0.5
        if comm == torch.float32:
            assert torch.allclose(src, total, atol=1e-6)
        else:
            bound = 3 * 2 ** -8 * total.abs().max().item()
            assert (src - total).abs().max().item() <= bound
            assert torch.equal(gbuf, local)        # the fp32 buffer is not overwritten with the sum
