"""Trainer — the reference's src/trainer.py surface (Trainer(model, args, device,
dataset, logger, processor), .train(), .eval(), .run_batch(), .load_ckpt())
re-built MI355X-first:

* one process per GPU (torchrun), RCCL all-reduce of flat gradient buckets
  overlapped with backward (deepfake_amd.ddp) instead of DataParallel
  (src/trainer.py:74-75);
* parameters / gradients in flat buffers with a bf16 compute shadow
  (deepfake_amd.params), fused SGD(momentum 0.9, weight decay) +
  CosineAnnealingLR (src/trainer.py:80-85) with the lr in device memory;
* BCELoss on the sigmoid output (src/trainer.py:88,132), accuracy
  (prob >= 0.5) == label (:142-144), gradient accumulation over accum_step
  micro-batches with the all-reduce only on the last one (:280-297);
* host<->device synchronisation only at log steps (the reference syncs every
  step at :133,136);
* optional HIP-graph capture of the whole step (TrainStep(graph=True)).
"""
import math
import os
import time

import torch
import torch.distributed as dist

from . import rng
from .ddp import GradBucketer, fr_last_id, recorder_on
from .optim import CosineAnnealingLR, FusedSGD
from .params import ParamStore
from .utils import AverageMeter, Logger


def pad_longest(waves):
    """The processor's padding='longest' (src/trainer.py:258): zero-pad every waveform of the batch to the
    longest one -> [B, S] fp32 (host)."""
    if torch.is_tensor(waves):
        return waves.float()
    arrs = [torch.as_tensor(w, dtype=torch.float32).reshape(-1) for w in waves]
    S = max(a.numel() for a in arrs)
    out = torch.zeros(len(arrs), S, dtype=torch.float32)
    for i, a in enumerate(arrs):
        out[i, :a.numel()] = a
    return out


def normalize_wave(w):
    """Wav2Vec2FeatureExtractor zero-mean / unit-variance (HF feature_extraction_wav2vec2.py:94-95) of every
    zero-padded row, whole row included (no attention mask, Q13) — on the GPU (dfk_wave_normalize)."""
    from . import kernels as K
    return K.wave_normalize(w)


def check_finite(loss, step, group=None, device="cpu"):
    """Failure detection at log steps (the only host sync of the loop): a NaN / Inf loss stops training with an
    error instead of stepping SGD on garbage.  The attention kernels are built without NaN semantics
    (build.py), so a diverging run is caught here, at the loss, not inside the kernels.
    Data-parallel (group given): the loss is rank-local while the gradients are averaged, so one rank's bad
    batch must not make that rank alone raise while the others block in the next bucket all-reduce until the
    RCCL watchdog fires — the non-finite flag is MAX-all-reduced and every rank raises at the same step."""
    bad = not math.isfinite(loss)
    if group is not None:
        flag = torch.tensor([1.0 if bad else 0.0], device=device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if flag.item() > 0 and not bad:
            raise FloatingPointError(f"non-finite training loss on another rank at optimizer step {step} "
                                     f"(this rank: {loss})")
    if bad:
        raise FloatingPointError(f"non-finite training loss {loss} at optimizer step {step}")
    return loss


def prepare_video(video, device, augment=False, generator=None, size=224):
    """Frames to the device: fp32 transform output as is; decoded uint8 RGB frames [B,T,H,W,3] transformed on
    the GPU -> [B,T,3,h,w] with the reference's torchvision transforms on PIL images (PIL semantics,
    media.frame_augment): eval (data/data_process.py:55-60) T.Resize(224) (shorter side; a no-op on 224 x 224
    frames, which then take the plain ToTensor + Normalize kernel) + ToTensor + Normalize; with augment the
    training transform (:62-69: Resize((224, 224)), RandomHorizontalFlip, RandomVerticalFlip, RandomRotation(90),
    drawn per frame in the reference's order, as it transforms every frame separately)."""
    from . import kernels as K
    from . import media
    v = video.to(device, non_blocking=True)
    if v.dtype != torch.uint8:
        return v
    H, W = v.shape[-3], v.shape[-2]
    if not augment:
        if min(H, W) == size:
            return K.frame_normalize(v)
        oh, ow = media.eval_size(H, W, size)
        return media.frame_augment(v, (ow, oh))
    n = v.numel() // (H * W * 3)
    flips, angles = media.draw_augment(n, generator)
    return media.frame_augment(v, (size, size), flips=flips, angles=angles)


def prepare_mel(audio, device, augment=False, generator=None, size=224):
    """The mel slot's input to the device: the normalised image as is; the uint8 grey image (the reference's
    cached JPEG, data_process.py:162) normalised on the GPU; a raw 22.05 kHz waveform [B, S] turned into the
    mel-spectrogram image on the GPU first (generate_mel_spectrogram, src/utils.py:63-87).  augment: the
    reference runs the mel JPEG through the same self.transform as the frames (data_process.py:162) — in training
    Resize((224, 224)) + flips + RandomRotation(90), one draw per image (media.frame_augment on the grey image)."""
    from . import media
    a = audio.to(device, non_blocking=True)
    if a.dtype != torch.uint8 and a.dim() == 2:
        a = media.mel_image(a)
    if a.dtype == torch.uint8:
        if augment:
            n = a.numel() // (a.shape[-2] * a.shape[-1])
            flips, angles = media.draw_augment(n, generator)
            return media.frame_augment(a, (size, size), flips=flips, angles=angles, grey=True)
        return media.gray_normalize(a)
    return a


class TrainStep:
    """fwd + BCE + bwd + gradient all-reduce + SGD for one micro-batch, optionally
    captured once into a HIP graph and replayed (inputs copied into static buffers).

    ``micro(feature, label, last, accum)`` is the gradient-accumulation form of
    src/trainer.py:280-297: loss / accum -> backward for every micro-batch; the
    non-final ones run under the bucketer's no_sync() (no all-reduce), the final
    one launches the overlapped bucket all-reduces over the accumulated sum, then
    SGD and zero_grad.  BatchNorm running statistics are re-broadcast from rank 0
    at the first micro-step of every optimizer step (§8e)."""

    def __init__(self, model, store, opt, bucketer, graph=False, parallel_branches=True):
        self.model, self.store, self.opt, self.bucketer = model, store, opt, bucketer
        if parallel_branches and hasattr(model, "parallel_branches") and torch.cuda.is_available() \
                and store.flat.is_cuda:
            model.parallel_branches = True
            bucketer.streams = model.branch_streams()
        self.lossF = torch.nn.BCELoss()
        self.graph_mode = graph
        self.graph = None
        self.static = None
        self.captured_overlap = None     # form of the captured step (None: not captured)
        self.captured_bn = False
        self.agraphs = None              # accumulation: (non-final micro-step, final micro-step) graphs
        self.first_micro = True
        if not bucketer.bn_buffers:
            bucketer.track_batchnorm(model)

    def _fwd_bwd(self, feature, label, scale=1.0, before_backward=None):
        rng.advance(self.store.flat.device)   # fresh dropout / DropPath / LayerDrop / SpecAugment draws
        prob = self.model(feature)
        loss = self.lossF(prob.float().reshape(-1), label.float().reshape(-1))
        if before_backward is not None:
            before_backward()
        (loss * scale if scale != 1.0 else loss).backward()
        if getattr(self.model, "parallel_branches", False):
            self.model.join_branches()
        return loss, prob

    def micro(self, feature, label, last, accum=1):
        """One micro-step of an accumulation window (eager, or replayed from the window's two graphs)."""
        if self.graph_mode and accum > 1:
            return self._micro_graphed(feature, label, last, accum)
        return self._micro_eager(feature, label, last, accum)

    def _micro_eager(self, feature, label, last, accum):
        if self.first_micro:
            self.bucketer.broadcast_bn()
            self.first_micro = False
        if not last:
            with self.bucketer.no_sync():
                loss, prob = self._fwd_bwd(feature, label, 1.0 / accum)
            return loss.detach(), prob.detach()
        loss, prob = self._fwd_bwd(feature, label, 1.0 / accum)
        fold = self._fold()
        fa = self.bucketer.finish(fold=fold)   # overlapped bucket all-reduces (hooks); the mean is taken by SGD
        self.opt.step(**fa)             # first call initialises the momentum buffer (torch SGD semantics)
        self.store.zero_grad()
        self.first_micro = True
        # detach: a live autograd graph would pin AccumulateGrad nodes to this stream (breaks capture)
        return loss.detach(), prob.detach()

    def _fold(self):
        """The fused SGD kernel takes the all-reduced sum and the 1 / world scale itself (no averaging pass)."""
        return isinstance(self.opt, FusedSGD)

    def eager(self, feature, label):
        return self._micro_eager(feature, label, True, 1)

    def __call__(self, feature, label):
        if not self.graph_mode:
            return self.eager(feature, label)
        if self.graph is None:
            loss, prob = self.eager(feature, label)   # initialises momentum, warms the allocator
            self._capture_step(feature, label)
            return loss, prob
        if not self.captured_bn:
            self.bucketer.broadcast_bn()
        self._load_static(feature, label)
        self.graph.replay()
        return self.static[2], self.static[3]

    def _micro_graphed(self, feature, label, last, accum):
        """Gradient accumulation with graphs (src/trainer.py:280-297 at --accum_step > 1): the non-final micro-step
        (fwd + bwd of loss / accum under no_sync) and the final one (the same, then the bucket all-reduces, SGD and
        the gradient zeroing that opens the next window) are captured as two graphs after one eager window, and
        each micro-step replays one of them.  BatchNorm statistics are broadcast eagerly at each window's start."""
        if self.agraphs is None:
            loss, prob = self._micro_eager(feature, label, last, accum)
            if last:
                self._capture_accum(feature, label, accum)
            return loss, prob
        if self.first_micro:
            self.bucketer.broadcast_bn()
            self.first_micro = False
        self._load_static(feature, label)
        g, outs = self.agraphs[1] if last else self.agraphs[0]
        g.replay()
        if last:
            self.first_micro = True
        return outs

    def input_buffers(self):
        """The replayed graph's input tensors ((video, mel, wave), label), or None before the capture.  A data
        loader that writes each batch into them in place (and passes them back to __call__) saves the per-step
        device-to-device copy into the graph's inputs (~0.2 GB at C2, B = 8)."""
        if self.static is None:
            return None
        return tuple(self.static[0]), self.static[1]

    def _load_static(self, feature, label):
        for s, x in zip(self.static[0], feature):
            if x is not s:   # already the graph's input (a loader writing in place): nothing to copy
                s.copy_(x, non_blocking=True)
        if label is not self.static[1]:
            self.static[1].copy_(label, non_blocking=True)

    # capture forms, tried in order (multi-GPU): (bucket all-reduces overlapped with backward, BatchNorm
    # running-stat broadcast inside the graph)
    FORMS = ((True, True), (False, True), (False, False))

    def _agree(self, ok):
        """All ranks commit to a capture form only if every rank captured it (a rank that fell back alone would
        issue a different collective sequence per step: deadlock or mis-reduction at the first replay)."""
        if not self.bucketer.enabled:
            return ok
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.store.flat.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.bucketer.group)
        return bool(flag.item())

    def _graph(self, body, forms):
        """Capture body(overlap, bn) -> outputs into a HIP graph under the first form every rank can capture.
        RCCL and the capture: the ProcessGroupNCCL watchdog thread queries the events of eager collectives
        until it retires them, and HIP refuses such a query once the RCCL stream joins a capture (the watchdog
        then aborts the process).  Every capture attempt therefore starts only after GradBucketer.drain has
        observed, through the flight recorder, that the watchdog retired every eager collective; the capture
        runs in thread-local mode so no other thread's legal call can invalidate it.
        Returns (graph, outputs, form) or (None, error, None)."""
        err = None
        if self.bucketer.enabled and not recorder_on():   # the same environment on every rank: all go eager
            return None, RuntimeError("TORCH_FR_BUFFER_SIZE unset: the RCCL watchdog cannot be observed idle"), None
        for overlap, bn in forms:
            # every failure below (drain timeout included) is local to this rank: it only marks the attempt
            # failed, so every rank still reaches the _agree all-reduce and all move to the next form together
            g, outs, ok = None, None, True
            try:
                self.bucketer.drain(self.bucketer.last_works)
            except RuntimeError as e:
                err, ok = e, False
            if ok:
                fr0 = fr_last_id() if self.bucketer.watched() else None
                self.bucketer.overlap = overlap
                self.bucketer.reset()
                self.store.uses.clear()   # a failed attempt may have left forward-use counts behind
                try:
                    g, outs = self._capture_once(body, overlap, bn)
                except RuntimeError as e:     # e.g. a collective the backend cannot capture in this form
                    err, ok, g = e, False, None
                    if fr0 is not None:       # its captured collectives never run: the drain must not wait on them
                        self.bucketer.fr_exclude.append((fr0, fr_last_id()))
                self.bucketer.overlap = True
                self.bucketer.reset()
            if not self._agree(ok):
                del g
                continue
            return g, outs, (overlap, bn)
        return None, err, None

    def _capture_once(self, body, overlap, bn):
        """One capture of body(overlap, bn) in thread-local mode on a side stream -> (graph, outputs); raises
        RuntimeError when the capture fails (the device is synchronised first)."""
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        try:
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    outs = body(overlap, bn)
        except RuntimeError:
            torch.cuda.synchronize()
            torch.cuda.current_stream().wait_stream(s)
            raise
        torch.cuda.current_stream().wait_stream(s)
        return g, outs

    def _step_body(self, static_in, static_label, accum):
        """The optimizer step's graph body: (zeroing,) BN broadcast, fwd + bwd, all-reduces, SGD."""
        # where the step graph zeroes the gradients (A/B): 0 at the start, 1 after the forward, 2 on a side stream
        # beside the forward (joined before the backward)
        zmode = int(os.environ.get("DFK_ZERO_MODE", "0")) if accum == 1 else 0

        def body(overlap, bn):
            join = None
            if accum == 1:
                if zmode == 0:
                    self.store.grad.zero_()
                elif zmode == 2:
                    zs = self._side_stream()
                    zs.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(zs):
                        self.store.grad.zero_()
                    join = lambda: torch.cuda.current_stream().wait_stream(zs)   # noqa: E731
                else:
                    join = self.store.grad.zero_
                self.store.zero_gates()
                if bn:
                    self.bucketer.broadcast_bn()
            l2, p2 = self._fwd_bwd(tuple(static_in), static_label, 1.0 / accum, before_backward=join)
            fold = self._fold()
            if overlap:
                fa = self.bucketer.finish(fold=fold)   # flush unused buckets, join the comm stream
            else:
                fa = self.bucketer.allreduce_all(fold=fold)
            self.opt.step(first=False, **fa)
            if accum > 1:                      # the next window starts from zero gradients and gates
                self.store.grad.zero_()
                self.store.zero_gates()
            return l2.detach(), p2.detach()
        return body

    def _side_stream(self):
        if getattr(self, "_zstream", None) is None:
            self._zstream = torch.cuda.Stream()
        return self._zstream

    def _fallback(self, err):
        self.graph_mode = False
        print(f"[deepfake_amd] HIP-graph capture failed ({err}); running the step eagerly", flush=True)
        self.store.zero_grad()

    def _capture_step(self, feature, label):
        """Capture the whole step — grad zeroing, BN broadcast, fwd, bwd, bucket all-reduces, SGD — as one graph.
        Multi-GPU: the bucket all-reduces are captured where the backward completes each bucket (on the comm
        stream, overlapping the rest of backward, §8e); if any rank cannot capture that form, every rank retries
        with one all-reduce pass after backward, then with the BN broadcast outside the graph, and only then do
        all ranks run eagerly."""
        self.static = [[x.clone() for x in feature], label.clone(), None, None]
        forms = self.FORMS if self.bucketer.enabled else ((False, False),)
        if os.environ.get("DFK_CAPTURE_OVERLAP") == "0":   # probes: only the one-pass forms
            forms = tuple(f for f in forms if not f[0])
        g, outs, form = self._graph(self._step_body(self.static[0], self.static[1], 1), forms)
        if g is None:
            return self._fallback(outs)
        self.graph = g
        self.static[2], self.static[3] = outs
        self.captured_overlap, self.captured_bn = form

    def _capture_accum(self, feature, label, accum):
        """The accumulation window's two graphs (after one eager window: momentum initialised)."""
        self.static = [[x.clone() for x in feature], label.clone(), None, None]

        def mid(overlap, bn):
            with self.bucketer.no_sync():
                l2, p2 = self._fwd_bwd(tuple(self.static[0]), self.static[1], 1.0 / accum)
            return l2.detach(), p2.detach()
        gm, outs_m, _ = self._graph(mid, ((False, False),))
        if gm is None:
            return self._fallback(outs_m)
        forms = tuple((o, False) for o in ((True, False) if self.bucketer.enabled else (False,)))
        gl, outs_l, form = self._graph(self._step_body(self.static[0], self.static[1], accum), forms)
        if gl is None:
            return self._fallback(outs_l)
        self.agraphs = ((gm, outs_m), (gl, outs_l))
        self.captured_overlap, self.captured_bn = form


class Trainer:
    def __init__(self, model, args, device, dataset, logger=None, processor=None, compute_dtype=None, graph=False):
        self.train_epochs = args.epochs
        self.device = device
        self.lr = args.learning_rate
        self.batch_size = args.batch_size
        self.modality = args.modality
        self.logger = logger or Logger(None)
        self.processor = processor
        self.model_save = args.model_save
        self.log_step = args.log_step
        self.start_epoch = 0
        self.accum_step = max(1, int(args.accum_step))
        self.augment = bool(getattr(args, "augment", False))
        self.dataset = dataset
        self.trainloader = dataset.train_dataloader()
        self.valloader = dataset.val_dataloader()
        dt = compute_dtype or (torch.bfloat16 if getattr(args, "dtype", "bf16") == "bf16" else torch.float32)
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        # device-side regulariser streams from --random_seed: per-rank element masks (dropout, DropPath,
        # SpecAugment), one shared stream for the LayerDrop coins (train.py:67 seed_torch seeds only torch)
        rng.manual_seed(int(getattr(args, "random_seed", 0)), self.rank)
        model.to(device)
        self.model_s = self.model = model
        self.store = ParamStore(model, dt)
        self.bucketer = GradBucketer(self.store, bucket_mb=getattr(args, "bucket_mb", 64.0),
                                     comm_dtype=torch.bfloat16 if getattr(args, "bucket_dtype", "fp32") == "bf16"
                                     else torch.float32)
        self.bucketer.broadcast_buffers(model)
        if self.bucketer.enabled:                      # identical replicas: parameters from rank 0
            dist.broadcast(self.store.flat, 0)
            self.store.refresh_shadow()
        self.optimizer = FusedSGD(self.store, args.learning_rate, momentum=0.9, weight_decay=args.l2_decacy)
        steps_per_epoch = max(1, int(len(self.trainloader) / self.accum_step))
        self.scheduler = CosineAnnealingLR(self.optimizer, T_max=self.train_epochs * steps_per_epoch)
        self.step_fn = TrainStep(model, self.store, self.optimizer, self.bucketer, graph=graph)
        self.lossF = torch.nn.BCELoss()
        n = sum(p.numel() for p in model.parameters())
        self.logger(f"model params: {n / 1e6:.3f} M ({n * 4 / 2 ** 20:.1f} MiB fp32)")

    def load_ckpt(self, args):
        """src/trainer.py:90-122: {'checkpoint': state_dict} with strict=False and
        'module.' stripping for single-modality runs; optimizer/epoch not restored."""
        path = args.fused_ckpt_path if self.modality == "fused" else (
            args.audio_ckpt_path if self.modality == "audio" else args.video_ckpt_path)
        ck = torch.load(path, map_location="cpu", weights_only=True)
        sd = ck["checkpoint"]
        if self.modality != "fused":
            sd = {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}
        self.model_s.load_state_dict(sd, strict=False)
        self.store.refresh_shadow()
        self.logger("Load Finetuned Model Succesfully")

    def save_ckpt(self, path, epoch):
        if self.rank == 0:
            torch.save({"epoch": epoch, "checkpoint": self.model_s.state_dict(),
                        "optimizer": self.optimizer.state_dict()}, path)

    def _features(self, feat):
        """src/trainer.py:250-262: the batch's features on the device, waveforms padded to the longest and
        normalised (the processor), frames normalised when they arrive as decoded uint8."""
        aug = self.augment and self.model.training
        if self.modality == "fused":
            wave = normalize_wave(pad_longest(feat["PAudio"]).to(self.device, non_blocking=True))
            return (prepare_video(feat["Video"], self.device, aug), prepare_mel(feat["Audio"], self.device, aug), wave)
        if self.modality == "paudio":
            return normalize_wave(pad_longest(feat).to(self.device, non_blocking=True))
        if self.modality == "video":
            return prepare_video(feat, self.device, aug)
        return prepare_mel(feat, self.device, aug)

    def _prep(self, batch):
        return self._features(batch[0]), batch[1].to(self.device, non_blocking=True)

    def submit(self, dataloader=None, path="prediction.csv"):
        """Inference over the test split (src/submit.py:79-120, SubmitCtl.submit): appends
        'filename,probability' rows to `path`; returns {filename: probability}."""
        dataloader = dataloader or self.dataset.test_dataloader()
        self.model.eval()
        res = {}
        with torch.no_grad(), open(path, "a") as f:
            for iter_id, (feat, names) in enumerate(dataloader):
                out = self.model(self._features(feat)).float().reshape(-1).cpu()
                for name, v in zip(names, out.numpy()):
                    f.write("{0},{1}\n".format(name, v))
                    res[name] = float(v)
                if iter_id % self.log_step == 0:
                    self.logger("|step {:4d} |total {:4d}| Rate% {:.3f}".format(iter_id, len(dataloader),
                                                                               iter_id / len(dataloader) * 100))
        self.logger("Test Score Prediction Done")
        self.model.train()
        return res

    def run_batch(self, feature, label, gpu_log=None):
        """Forward + loss + accuracy (src/trainer.py:124-148); no host sync here."""
        out = self.model(feature)
        loss = self.lossF(out.float().reshape(-1), label.float().reshape(-1))
        with torch.no_grad():
            acc = ((out.reshape(-1) >= 0.5) == label.reshape(-1).to(torch.bool)).float().mean()
        return {"loss": loss, "acc": acc}

    def eval(self, dataloader, epoch, t, lr, val_loss_draw=None, gpu_log=None):
        stat = AverageMeter()
        self.model.eval()
        with torch.no_grad():
            for batch in dataloader:
                feature, label = self._prep(batch)
                r = self.run_batch(feature, label)
                if t % self.log_step == 0:
                    self.logger("| epoch {:2d} | step {:4d} | lr {:.4E} | Val Loss {:3.5f} | Val Acc {:1.5f} ".format(
                        epoch, t, lr, r["loss"].item(), r["acc"].item()))
                stat.update(r["loss"].item())
                t += 1
        self.logger(f"Phase:val, Avg Loss:{stat.avg}")
        self.model.train()
        return t

    def train(self):
        t = 0
        stat = AverageMeter()
        self.logger("[INFO] Start training, lr = {:.6f}".format(self.optimizer.param_groups[0]["lr"]))
        for epoch in range(self.start_epoch, self.train_epochs + 1):
            self.model.train()
            self.store.zero_grad()
            t0 = time.time()
            for iter_id, batch in enumerate(self.trainloader):
                feature, label = self._prep(batch)
                last = (iter_id + 1) % self.accum_step == 0
                if self.accum_step == 1:
                    loss, prob = self.step_fn(feature, label)
                else:
                    loss, prob = self.step_fn.micro(feature, label, last, self.accum_step)
                if last:
                    t += 1
                    self.scheduler.step()
                    if t % self.log_step == 0:
                        li = loss.item()
                        check_finite(li, t, (self.bucketer.group or dist.group.WORLD) if self.bucketer.enabled
                                     else None, self.store.grad.device)
                        stat.update(li)
                        dt = time.time() - t0
                        self.logger("| epoch {:2d} | step {:4d} | lr {:.4E} | Train Loss Avg {:3.5f} | clips/s {:.2f}"
                                    .format(epoch, t, self.optimizer.param_groups[0]["lr"], stat.avg,
                                            self.log_step * self.accum_step * self.batch_size / max(dt, 1e-9)))
                        t0 = time.time()
                    if self.model_save and (t + 1) % self.model_save == 0 and last:
                        os.makedirs("checkpoints", exist_ok=True)
                        self.save_ckpt(f"./checkpoints/VST_deepfake_modality{self.modality}_batch{self.batch_size}"
                                       f"_epoch{epoch}_step{t}.pth", epoch)
            self.logger(f"Phase:train, Avg Loss:{stat.avg}")
            stat.reset()
            if self.valloader is not None:
                t = self.eval(self.valloader, epoch, t, self.optimizer.param_groups[0]["lr"])
