#!/usr/bin/env python
"""bench.py — train clips/s of the north-star fused deepfake model on MI355X.

Workload (BASELINE.json configs[1], "C2"): Video Swin-T (depths 2,2,6,2, window
8x7x7, patch 2x4x4) over 32x224x224 clips + SwinV2 mel branch (128; 2,2,18,2)
over a 224x224 mel image + wav2vec2-base over 4 s @ 16 kHz + FusionModel head;
B=8 clips per GPU; bf16 compute (fp32 master weights, fp32 softmax/LN stats);
one step = forward + BCE + backward + RCCL gradient all-reduce + fused SGD
(momentum 0.9, wd) with the reference's training regularisers on (VST DropPath
0.2, SwinV2 DropPath 0.1, wav2vec2 feat-proj / hidden / activation / attention
dropout 0.1, LayerDrop 0.1, SpecAugment mask_time_prob 0.05, Audio2D and head
dropout 0.1; --deterministic turns them off) — the whole step captured in one HIP graph and replayed
(the first warm-up step runs eagerly and captures; --eager replays nothing), with
the video / mel / waveform trunks on three HIP streams inside the graph.
Inputs are synthetic, generated on device and resident in HBM.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints ONE JSON line (value = whole-job clips/s, max step time over ranks).
"""
import argparse
import json
import math
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

# Before any process group exists: RCCL work events are not drawn from torch's event cache, so the bucket
# all-reduces captured into the step's HIP graph never share an event with an eager collective the
# ProcessGroupNCCL watchdog is still polling (with the cache on, the watchdog's query of a
# capture-recorded event aborts the process: tools/ddp_graph_probe.py).
os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
# The flight recorder lets the capture observe that the watchdog retired every eager collective
# (deepfake_amd.ddp.watchdog_idle) instead of guessing with a sleep.
os.environ.setdefault("TORCH_FR_BUFFER_SIZE", "256")

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "train clips/sec (32x224x224 video + 16kHz audio) at 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="c2")
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp8"],
                   help="fp8: bf16 compute with the video trunk's stage-3/4 Linears on MX-fp8 GEMMs (C4's fp8 path)")
    p.add_argument("--eager", action="store_true", help="run the step eagerly instead of replaying its HIP graph")
    p.add_argument("--deterministic", action="store_true", help="regularisers off (the parity setting)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-steps", type=int, default=3)
    p.add_argument("--cpu-threads", type=int, default=None, help="torch threads of the CPU baseline (default: every "
                   "CPU in this process's affinity mask within its cgroup CPU quota, BASELINE.md §4)")
    p.add_argument("--roofline-iters", type=int, default=20)
    return p.parse_args()


def synthetic_batch(cfg, B, device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    video = torch.randn(B, cfg["T"], 3, cfg["H"], cfg["W"], device=device, generator=g)
    mel = torch.randn(B, 3, 224, 224, device=device, generator=g)
    wave = torch.randn(B, int(16000 * cfg["seconds"]), device=device, generator=g)
    wave = (wave - wave.mean(1, keepdim=True)) / torch.sqrt(wave.var(1, keepdim=True, unbiased=False) + 1e-7)
    label = (torch.rand(B, device=device, generator=g) < 0.5).float()
    return (video, mel, wave), label


def time_kernel(fn, iters):
    """Average duration of fn's launches between HIP events on the current stream."""
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e-3   # seconds per launch


ROOFLINE_KERNEL = "wattn_fwd6_kernel<false>"
ROOFLINE_PMC = os.path.join(HERE, "profiles", "r6", "r6_wattn_fwd_pmc.json")   # tools/gpu_round6.sh


def stage1_geometry(cfg):
    """Stage-1 attention geometry of this config's video trunk: (C, heads, window, shift, (D, H, W))."""
    v = cfg["vst"]
    C, heads = v["embed_dim"], v["num_heads"][0]
    dims = (cfg["T"] // 2, cfg["H"] // 4, cfg["W"] // 4)
    win = tuple(min(w, d) for w, d in zip(v["window_size"], dims))
    shift = tuple(0 if d <= w else w // 2 for w, d in zip(v["window_size"], dims))
    return C, heads, win, shift, dims


def roofline_case(cfg, B, dt):
    """Dominant MFMA kernel: the stage-1 shifted-window attention core of this config's video backbone
    (B clips; Swin-T / Swin-B: window 8x7x7 = 392 tokens, 3 / 4 heads x 32, shift (4,3,3), relative-position
    bias).  Returns (launch fn, algorithmic FLOPs per launch = 4 * windows * heads * N^2 * hd, i.e. QK^T and
    PV, description)."""
    from deepfake_amd import kernels as K
    C, heads, win, shift, (D, H, W) = stage1_geometry(cfg)
    hd = C // heads
    rows = B * D * H * W
    g = torch.Generator(device="cuda").manual_seed(7)
    qkv = torch.randn(rows, 3 * C, device="cuda", generator=g).to(dt)
    nW = -(-D // win[0]) * -(-H // win[1]) * -(-W // win[2])
    N = win[0] * win[1] * win[2]
    flops = 4.0 * B * nW * heads * N * N * hd
    L = (2 * win[0] - 1) * (2 * win[1] - 1) * (2 * win[2] - 1)
    rpb = torch.randn(L, heads, device="cuda", generator=g) * 0.02
    out = torch.empty(rows, C, device="cuda", dtype=dt)
    args = (qkv, qkv[:, C:], qkv[:, 2 * C:], 3 * C, (B, D, H, W), win, win, shift, heads, hd, hd ** -0.5)
    # the bf16 score-bias tiles (dfk_wattn_table, a separate launch) are built once: the timed launch is the
    # attention kernel alone, the one rocprofv3 lists as wattn_fwd6_kernel<false> (16x16x32 tiles)
    _, _, tab = K.wattn_fwd(*args, rpb=rpb, out=out, return_table=True)

    def run():
        K.wattn_fwd(*args, rpb=rpb, out=out, need_lse=True, tab=tab)
    desc = (f"stage-1 SW-MSA core, {N}-token windows, {heads} heads x {hd}, shift {'x'.join(map(str, shift))}, RPB, "
            f"{B * nW * heads} window-heads")
    return run, flops, desc


def pmc_traffic():
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 PMC
    passes (tools/roofline_pmc.py: FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE)."""
    try:
        with open(ROOFLINE_PMC) as f:
            d = json.load(f)
        if d.get("kernel") != ROOFLINE_KERNEL:   # counters of another kernel say nothing about this one
            return None, None
        return d["bytes_per_launch"], os.path.relpath(ROOFLINE_PMC, HERE)
    except (OSError, KeyError, ValueError):
        return None, None


CONV3D_KERNEL = "pe_fwd_kernel<6>"
CONV3D_INSTEP = os.path.join(HERE, "profiles", "r6", "r6_conv3d_instep.json")   # tools/gpu_round6.sh


def conv3d_in_step():
    """The same kernel's launches INSIDE the replayed training step, from the committed rocprofv3 kernel trace of
    this bench command (tools/pe_instep.py separates them from the isolated loop's launches)."""
    try:
        with open(CONV3D_INSTEP) as f:
            d = json.load(f)["in_step"]
        return {"launches": d["launches"], "median_us": d["median_us"], "achieved_gbs": d["achieved_gbs_median"],
                "frac": d["frac_median"], "source": os.path.relpath(CONV3D_INSTEP, HERE)}
    except (OSError, KeyError, ValueError, TypeError):
        return None


def conv3d_roofline(cfg, B, iters, nbuf=3, instep=False):
    """The whole Conv3D patch embed (PatchEmbed3D pad + Conv3d(3->96, 2x4x4) + LayerNorm(96),
    video_swin_transformer.py:446-458) as the ONE fused launch the training step runs
    (dfk_patch_embed_fwd): the fp32 clip batch [B,T,3,H,W] is read once, the normalised bf16 tokens
    [tokens, 96] and their fp32 LN statistics (mean, rstd) are written once.  Algorithmic bytes per launch
    = B*T*3*H*W*4 + tokens*(96*2 + 8) (29.3 MB per 32x224x224 clip).  Timed COLD: `nbuf` distinct clip
    batches (and outputs) are rotated so the working set (3 x 231 MB at B=8) exceeds the 256 MiB Infinity
    Cache and every launch streams from HBM."""
    from deepfake_amd import kernels as K
    g = torch.Generator(device="cuda").manual_seed(5)
    vids = [torch.randn(B, cfg["T"], 3, cfg["H"], cfg["W"], device="cuda", generator=g) for _ in range(nbuf)]
    C = cfg["vst"]["embed_dim"]
    w = (torch.randn(C, 96, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    b, lw, lb = (torch.randn(C, device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
    tokens = B * (cfg["T"] // 2) * (cfg["H"] // 4) * (cfg["W"] // 4)
    nbytes = vids[0].numel() * 4 + tokens * (C * 2 + 8)
    state = {"i": 0}

    def run():
        state["i"] = (state["i"] + 1) % nbuf
        K.patch_embed_fwd(vids[state["i"]], "btchw", w, b, lw, lb, 1e-5)
    t = time_kernel(run, iters)
    achieved = nbytes / t / 1e9
    return {"kernel": CONV3D_KERNEL + f" (fused pad + Conv3d 2x4x4 -> {C} + LayerNorm of the clip batch, cold)",
            "bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 4), "bytes_per_launch": nbytes, "avg_launch_ms": round(t * 1e3, 4),
            "timing": f"HIP events over {iters} launches rotating {nbuf} clip batches (working set > Infinity Cache)",
            "in_step": conv3d_in_step() if instep else None}


ATTN_BWD_KERNELS = "wattn_bwd4_kernel + drpb_from_ds_kernel + drpb_reduce_kernel"


def attn_bwd_roofline(cfg, B, dt, iters):
    """The stage-1 shifted-window attention BACKWARD of the same launch as `roofline` (WindowAttention3D.forward's
    autograd, video_swin_transformer.py:142-173): dQ, dK, dV and the relative-position-bias gradient dRPB, i.e.
    the two-pass backward kernel (its dK/dV pass writes the window groups' summed dS^T slabs) plus the two dRPB
    launches (binning the slabs, reducing the partial rows).
    Algorithmic FLOPs = 10 * window-heads * N^2 * hd (dP = dO V^T, dV = P^T dO, dS -> dQ = dS K, dK = dS^T Q, plus the
    recomputed S = Q K^T); the dRPB binning is counted as no FLOPs."""
    from deepfake_amd import kernels as K
    C, heads, win, shift, (D, H, W) = stage1_geometry(cfg)
    hd = C // heads
    rows = B * D * H * W
    g = torch.Generator(device="cuda").manual_seed(8)
    qkv = torch.randn(rows, 3 * C, device="cuda", generator=g).to(dt)
    nW = -(-D // win[0]) * -(-H // win[1]) * -(-W // win[2])
    N = win[0] * win[1] * win[2]
    L = (2 * win[0] - 1) * (2 * win[1] - 1) * (2 * win[2] - 1)
    rpb = torch.randn(L, heads, device="cuda", generator=g) * 0.02
    args = (qkv, qkv[:, C:], qkv[:, 2 * C:], 3 * C, (B, D, H, W), win, win, shift, heads, hd, hd ** -0.5)
    out, lse, tab = K.wattn_fwd(*args, rpb=rpb, return_table=True)
    dout = torch.randn(rows, C, device="cuda", generator=g).to(dt)
    dqkv = torch.empty_like(qkv)
    drpb = torch.zeros_like(rpb)
    fa = (qkv, qkv[:, C:], qkv[:, 2 * C:], out, lse, 3 * C, (B, D, H, W), win, win, shift, heads, hd, hd ** -0.5,
          rpb, None)

    def run():
        K.wattn_bwd(fa, dout, dqkv, dqkv[:, C:], dqkv[:, 2 * C:], 3 * C, drpb=drpb, tab=tab)
    t = time_kernel(run, iters)
    flops = 10.0 * B * nW * heads * N * N * hd
    ach = flops / t / 1e12
    # the same launch with 4 windows per workgroup (the isolated kernel's best; the step runs faster at the default 8,
    # profiles/attn/r6_bwd4_group_sweep.txt) and without dRPB (the backward kernel alone, no slab writes)
    K.wattn_bwd_policy(group=4)
    try:
        t4 = time_kernel(run, iters)
    finally:
        K.wattn_bwd_policy(group=0)
    t0 = time_kernel(lambda: K.wattn_bwd(fa, dout, dqkv, dqkv[:, C:], dqkv[:, 2 * C:], 3 * C, drpb=None, tab=tab), iters)
    return {"kernel": ATTN_BWD_KERNELS + f" (stage-1 SW-MSA backward with dRPB, {N}-token windows, {heads} heads x "
            f"{hd}, {B * nW * heads} window-heads)", "bound": "mfma", "achieved": round(ach, 2),
            "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4),
            "flops_per_launch": flops, "avg_launch_ms": round(t * 1e3, 4),
            "group4": {"avg_launch_ms": round(t4 * 1e3, 4), "frac": round(flops / t4 / 1e12 / PEAK_BF16_TFLOPS, 4)},
            "no_drpb": {"avg_launch_ms": round(t0 * 1e3, 4), "frac": round(flops / t0 / 1e12 / PEAK_BF16_TFLOPS, 4)},
            "timing": f"HIP events over {iters} calls of the three launches (default: 8 windows per workgroup)"}


def roofline(cfg, B, dt, iters, pmc=True):
    run, flops, desc = roofline_case(cfg, B, dt)
    t = time_kernel(run, iters)
    achieved = flops / t / 1e12
    traffic, src = pmc_traffic() if pmc else (None, None)
    return {"kernel": ROOFLINE_KERNEL + f" ({desc})",
            "bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
            "traffic_source": src, "flops_per_launch": flops, "avg_launch_ms": round(t * 1e3, 4)}


GEMM_KERNEL = "gemm_dma_kernel<32|64, N, N, 2>"


def gemm_bound(flops, nbytes, t, peak_tflops):
    """Label a GEMM launch by its arithmetic intensity against the ridge of its dtype (peak FLOP/s over the 8 TB/s
    HBM peak): below the ridge it is HBM-bound and its fraction is bytes / time over HBM peak, above it MFMA-bound."""
    ridge = peak_tflops * 1e12 / (PEAK_HBM_GBS * 1e9)
    intensity = flops / nbytes
    if intensity < ridge:
        ach = nbytes / t / 1e9
        return {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(ach / PEAK_HBM_GBS, 4), "tflops": round(flops / t / 1e12, 2),
                "intensity_flop_per_byte": round(intensity, 1), "ridge_flop_per_byte": round(ridge, 1)}
    ach = flops / t / 1e12
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": peak_tflops, "unit": "TFLOP/s",
            "frac": round(ach / peak_tflops, 4), "intensity_flop_per_byte": round(intensity, 1),
            "ridge_flop_per_byte": round(ridge, 1)}


PEAK_FP8_TFLOPS = 5000.0       # MI355X dense fp8 (block-scaled MX e4m3) MFMA (MI355X_MICROARCH.md)
MX_GEMM_KERNEL = "gemm_mx_kernel<64, 2, 2, 2, true>"


def gemm_roofline(cfg, B, iters, fp8=False):
    """The step's largest Linear by time on the MFMA path: the video trunk's stage-3 Mlp.fc1 forward
    (video_swin_transformer.py Mlp, src/utils.py:254-256) with its fused bias + GELU epilogue that also
    saves the pre-activation — tokens = B * (T/2) * (H/16) * (W/16) rows, 4C -> 16C (Swin-T 384 -> 1536,
    Swin-B 512 -> 2048).  Algorithmic FLOPs per launch = 2 * M * N * K (the epilogue's elementwise work is
    not counted)."""
    from deepfake_amd import kernels as K
    g = torch.Generator(device="cuda").manual_seed(9)
    M = B * (cfg["T"] // 2) * (cfg["H"] // 16) * (cfg["W"] // 16)
    Kd = 4 * cfg["vst"]["embed_dim"]
    N = 4 * Kd
    x = torch.randn(M, Kd, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device="cuda", generator=g) * Kd ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.empty_like(out)
    trunk = "Swin-B" if cfg["vst"]["embed_dim"] == 128 else "Swin-T"
    flops = 2.0 * M * N * Kd
    if fp8:   # the step's MX-fp8 fc1: e4m3 operands with E8M0 block scales, GELU epilogue + MX copy of h for fc2
        xq, wq = K.mx_quant(x), K.mx_quant(w.float())

        def run_mx():
            K.gemm_mx(xq, wq, bias=b, out=out, act=1, aux=aux, mx_out=True)
        t = time_kernel(run_mx, iters)
        nbytes = M * Kd * (1 + 1 / 32) + N * Kd * (1 + 1 / 32) + M * N * (2 + 2 + 1 + 1 / 32)
        return dict({"kernel": MX_GEMM_KERNEL + f" ({trunk} stage-3 Mlp.fc1 fwd on MX-fp8, [{M},{Kd}]x[{Kd},{N}] + "
                     "bias + GELU, pre-activation saved, h also written quantised for fc2)"},
                    **gemm_bound(flops, nbytes, t, PEAK_FP8_TFLOPS), flops_per_launch=flops,
                    bytes_per_launch=round(nbytes), avg_launch_ms=round(t * 1e3, 4))

    def run():
        K.linear(x, w, b, out=out, act=1, aux=aux)
    t = time_kernel(run, iters)
    nbytes = (M * Kd + 2 * M * N + N * Kd) * 2
    return dict({"kernel": GEMM_KERNEL + f" ({trunk} stage-3 Mlp.fc1 fwd, [{M},{Kd}]x[{Kd},{N}] + bias + GELU, "
                 "pre-activation saved)"}, **gemm_bound(flops, nbytes, t, PEAK_BF16_TFLOPS), flops_per_launch=flops,
                bytes_per_launch=nbytes, avg_launch_ms=round(t * 1e3, 4))


DW_KERNEL = "gemm_dma_kernel<64, 2, 2, true, true, 2, true, false>"


def dw_roofline(cfg, B, iters):
    """The step's largest weight-gradient launch: the video trunk's stage-1 Mlp.fc1 dW with its fused bias gradient
    (src/utils.py:254-256 backward): dW[4C, C] += dy[tokens, 4C]^T x[tokens, C], db[4C] += colsum(dy), tokens =
    B * (T/2) * (H/4) * (W/4) (401k at C2), split over the tokens with fp32 atomics (kernels.linear_dw).  K = C is
    small, so the launch is HBM-bound: algorithmic bytes = tokens * 5C * 2 (dy and x read once, bf16) + the fp32
    dW / db read-modify-write."""
    from deepfake_amd import kernels as K
    g = torch.Generator(device="cuda").manual_seed(10)
    C = cfg["vst"]["embed_dim"]
    M = B * (cfg["T"] // 2) * (cfg["H"] // 4) * (cfg["W"] // 4)
    x = torch.randn(M, C, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(M, 4 * C, device="cuda", generator=g).to(torch.bfloat16)
    dw = torch.zeros(4 * C, C, device="cuda")
    db = torch.zeros(4 * C, device="cuda")

    def run():
        K.linear_dw(dy, x, dw, db=db)
    t = time_kernel(run, iters)
    nbytes = M * 5 * C * 2 + (4 * C * C + 4 * C) * 8
    achieved = nbytes / t / 1e9
    return {"kernel": DW_KERNEL + f" (stage-1 Mlp.fc1 weight + bias gradient, [{M},{4 * C}]^T x [{M},{C}], token split, "
            "fp32 atomics)", "bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 4), "bytes_per_launch": nbytes,
            "flops_per_launch": 2.0 * M * 4 * C * C, "avg_launch_ms": round(t * 1e3, 4)}


def _cpu_train_rate(cfg_name, B, steps):
    """Median seconds per fp32 CPU train step (fwd + BCE + bwd + SGD, train-mode BatchNorm) of the oracle."""
    from oracle import fusion as OF
    from oracle.fill import synthetic_inputs
    from deepfake_amd.models.fused import CONFIGS, W2V_CONFIG
    cfg = CONFIGS[cfg_name]
    m = OF.build_fused(cfg, W2V_CONFIG)
    m.train()
    opt = torch.optim.SGD(m.parameters(), lr=1e-4, momentum=0.9, weight_decay=0.05)
    video, mel, wave, label = synthetic_inputs(B, cfg["T"], cfg["H"], cfg["W"], cfg["seconds"], seed=1234)
    times = []
    for i in range(steps + 1):
        t0 = time.time()
        opt.zero_grad()
        p = m((video, mel, wave))
        loss = torch.nn.BCELoss()(p.reshape(-1), label)
        loss.backward()
        opt.step()
        if i > 0:
            times.append(time.time() - t0)
    return statistics.median(times)


def usable_cpus():
    """CPUs this process may actually use: its affinity mask, capped by the cgroup CPU quota (cpu.max) and by
    OMP_NUM_THREADS when the launcher sets it.  On the
    GPU box the mask lists 256 CPUs but the quota is 16 per GPU: the C2 oracle step took 5.7 s at 16 torch
    threads, 10.4 s at 64 and did not finish in 180 s at 256 (profiles/fp8/r4_mx_lane_map_probe.txt)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, math.ceil(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")   # the job's thread budget, when its launcher states one
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def cpu_baseline(cfg_name, steps, threads=None):
    """the oracle (CPU restatement of the reference, pinned to the reference's golden
    vectors) timed on the host cores: C1 and C2 at B=2, train-mode BatchNorm, one warm-up step then the
    median of `steps` train steps.  value = the C2 rate (the metric's workload)."""
    cores = len(os.sched_getaffinity(0))   # host CPUs this process may run on
    threads = usable_cpus() if threads is None else threads   # every CPU this process may use
    torch.set_num_threads(threads)
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    t1 = _cpu_train_rate("c1", 2, steps)
    t2 = _cpu_train_rate(cfg_name, 2, steps)
    return {"value": round(2.0 / t2, 4), "unit": "clips/s", "cores": threads, "threads": threads,
            "affinity_cpus": cores, "kind": "port",
            "c1_clips_per_s": round(2.0 / t1, 3), "cpu_model": cpu_model,
            "sample": f"oracle fp32 CPU train step (train-mode BN) at B=2: {cfg_name.upper()} {t2:.2f} s/step, "
                      f"C1 {t1:.3f} s/step; median of {steps} steps after 1 warm-up, {threads} torch threads = the CPUs "
                      f"usable under the cgroup quota ({cores} in the affinity mask)"}


def workload_name(name, cfg):
    v = cfg["vst"]
    trunk = "Swin-B" if v["embed_dim"] == 128 else "Swin-T"
    ckpt = ", activation-checkpointed video trunk" if v.get("use_checkpoint") else ""
    return (f"{name.upper()}: {trunk} video {cfg['T']}x{cfg['H']}x{cfg['W']} (window {'x'.join(map(str, v['window_size']))}) + "
            f"SwinV2 mel 224 + wav2vec2-base {cfg['seconds']}s@16kHz + FusionModel, full train step{ckpt}")


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16

    from deepfake_amd.ddp import GradBucketer
    from deepfake_amd.models.fused import CONFIGS, build_fused
    from deepfake_amd.optim import FusedSGD
    from deepfake_amd.params import ParamStore
    from deepfake_amd.trainer import TrainStep
    from deepfake_amd import rng

    cfg = CONFIGS[a.config]
    torch.manual_seed(1234)
    rng.manual_seed(1234, rank)
    model = build_fused(cfg, compute_dtype=dt, regularize=not a.deterministic, fp8=a.dtype == "fp8").to(device)
    model.train()
    store = ParamStore(model, dt)
    bucketer = GradBucketer(store, bucket_mb=64.0)
    if bucketer.enabled:
        dist.broadcast(store.flat, 0)
        store.refresh_shadow()
    opt = FusedSGD(store, lr=1e-4, momentum=0.9, weight_decay=1e-3)
    step = TrainStep(model, store, opt, bucketer, graph=not a.eager)
    feature, label = synthetic_batch(cfg, a.batch, device, 1234 + rank)

    for _ in range(max(a.warmup, 1)):
        loss, _ = step(feature, label)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss, _ = step(feature, label)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    lossv = float(loss.item())
    clips = world * a.batch * a.steps
    value = clips / el

    # committed counter / trace files describe the C2 bench command only: other configs report none
    c2 = a.config == "c2" and a.batch == 8
    roof = roofline(cfg, a.batch, dt, a.roofline_iters, pmc=c2) if rank == 0 else None
    roof_conv = conv3d_roofline(cfg, a.batch, a.roofline_iters, instep=c2) if rank == 0 else None
    roof_gemm = gemm_roofline(cfg, a.batch, a.roofline_iters, fp8=a.dtype == "fp8") if rank == 0 else None
    roof_dw = dw_roofline(cfg, a.batch, a.roofline_iters) if rank == 0 else None
    roof_bwd = attn_bwd_roofline(cfg, a.batch, dt, a.roofline_iters) if rank == 0 else None
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            cpu = cpu_baseline(a.config, a.cpu_steps, a.cpu_threads)
        except Exception as e:  # noqa: BLE001 — the baseline must not hide the measured line
            cpu = {"value": None, "unit": "clips/s", "cores": None, "kind": "port", "sample": f"failed: {e!r}"}
    if rank == 0:
        train_gflop = {"c1": 44.5, "c2": 790.2, "c4": 1951.0, "c5": 1590.0}.get(a.config)
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "clips/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": a.dtype, "data": "synthetic (device-resident, seeded)",
            "config": {"workload": workload_name(a.config, cfg),
                       "global_batch": world * a.batch, "per_gpu_batch": a.batch,
                       "parallelism": f"dp{world}", "hip_graph": step.graph is not None,
                       "captured_overlap": step.captured_overlap, "captured_bn_broadcast": step.captured_bn,
                       "branch_streams": 3,
                       "regularisers": not a.deterministic, "loss": round(lossv, 5)},
            "model_tflops_per_gpu": round(value / world * train_gflop / 1e3, 2) if train_gflop else None,
            "roofline": roof, "roofline_attn_bwd": roof_bwd, "roofline_conv3d": roof_conv, "roofline_gemm": roof_gemm,
            "roofline_dw": roof_dw,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
