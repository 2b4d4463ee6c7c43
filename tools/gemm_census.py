"""Census of every dfk_gemm launch in one C2 training step (B=8, bf16): shape, operand form and
HIP-event time per call, grouped and sorted by total time.  Also times the other kernel wrappers
(attention, LayerNorm, ...) per call site so the step's time splits by op.

    python tools/gemm_census.py [--config c2] [--batch 8]
"""
import argparse
import collections
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepfake_amd import kernels as K  # noqa: E402

REC = collections.defaultdict(lambda: [0, 0.0, 0.0])   # key -> [calls, ms, gflop]


def timed(name, fn, flop_fn=None):
    def wrap(*a, **k):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn(*a, **k)
        e.record()
        e.synchronize()
        key = name(*a, **k) if callable(name) else name
        rec = REC[key]
        rec[0] += 1
        rec[1] += s.elapsed_time(e)
        rec[2] += flop_fn(*a, **k) / 1e9 if flop_fn else 0.0
        return r
    return wrap


def gemm_key(a, a_ld, a_kmajor, b, b_ld, b_kmajor, M, N, Kd, c, ldc, **kw):
    form = ("T" if a_kmajor else "N") + ("T" if b_kmajor else "N")
    extra = []
    for f in ("bias", "residual", "aux", "rowsum"):
        if kw.get(f) is not None:
            extra.append(f)
    if kw.get("act"):
        extra.append(f"act{kw['act']}")
    if kw.get("atomic"):
        extra.append("atomic")
    if kw.get("splitk", 1) > 1:
        extra.append(f"sk{kw['splitk']}")
    if kw.get("a_conv") or kw.get("b_conv"):
        extra.append("conv")
    nz = kw.get("nz", (1, 1))
    return f"gemm {form} M={M} N={N} K={Kd} nz={nz[0] * nz[1]} {'+'.join(extra)}"


def gemm_flop(a, a_ld, a_kmajor, b, b_ld, b_kmajor, M, N, Kd, c, ldc, **kw):
    nz = kw.get("nz", (1, 1))
    return 2.0 * M * N * Kd * nz[0] * nz[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    from bench import synthetic_batch
    from deepfake_amd.ddp import GradBucketer
    from deepfake_amd.models.fused import CONFIGS, build_fused
    from deepfake_amd.optim import FusedSGD
    from deepfake_amd.params import ParamStore
    from deepfake_amd.trainer import TrainStep
    cfg = CONFIGS[a.config]
    dt = torch.bfloat16
    model = build_fused(cfg, compute_dtype=dt).cuda()
    model.train()
    store = ParamStore(model, dt)
    step = TrainStep(model, store, FusedSGD(store, 1e-4, 0.9, 1e-3), GradBucketer(store),
                     parallel_branches=False)   # one stream: per-call events time only that call
    feat, label = synthetic_batch(cfg, a.batch, torch.device("cuda"), 1)
    for _ in range(2):
        step(feat, label)
    torch.cuda.synchronize()
    K.gemm = timed(gemm_key, K.gemm, gemm_flop)
    for n in ("wattn_fwd", "wattn_bwd", "layernorm_fwd", "layernorm_bwd", "patch_im2col", "patch_merge", "rowmean",
              "w2v_conv0_fwd", "w2v_conv0_bwd", "gelu_bwd", "colsum", "sgd_step", "cast"):
        setattr(K, n, timed(n, getattr(K, n)))
    t0 = time.time()
    step(feat, label)
    torch.cuda.synchronize()
    wall = time.time() - t0
    tot = sum(v[1] for v in REC.values())
    print(f"synchronised step wall {wall * 1e3:.1f} ms; timed kernels {tot:.1f} ms")
    gem = sum(v[1] for k, v in REC.items() if k.startswith("gemm"))
    gfl = sum(v[2] for k, v in REC.items() if k.startswith("gemm"))
    print(f"gemm total {gem:.2f} ms, {gfl:.0f} GFLOP -> {gfl / gem:.0f} TFLOP/s")
    for k, (n, ms, gf) in sorted(REC.items(), key=lambda kv: -kv[1][1]):
        tf = f"{gf / ms:7.0f} TF/s" if gf else ""
        print(f"{ms:8.3f} ms {n:4d}x {ms / n * 1e3:8.1f} us {tf}  {k}")


if __name__ == "__main__":
    main()
