"""Throughput of the training input transform (--augment: data_process.py:62-69 — Resize((224, 224)), flips,
RandomRotation(90), ToTensor, Normalize per frame) against the step's rate, split into its parts: the host-side
draws (media.draw_augment), the host-side rotation matrices (media.pil_rotate_fixed per frame), the device
kernel on resident uint8 frames, and the whole trainer.prepare_video from pinned host frames (H2D included).
One "clip" = 32 frames, as in the C2 step.  Usage: python tools/augment_bench.py [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepfake_amd import media  # noqa: E402
from deepfake_amd.trainer import prepare_mel, prepare_video  # noqa: E402

B, T = 8, 32


def wall(fn, reps, sync=True):
    fn()
    if sync:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    if sync:
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    g = torch.Generator().manual_seed(0)
    n = B * T
    d = wall(lambda: media.draw_augment(n, g), reps, sync=False)
    _, angles = media.draw_augment(n, g)
    r = wall(lambda: [media.pil_rotate_fixed(a, 224, 224) for a in angles], reps, sync=False)
    print(f"host: draw_augment {n} frames {d*1e3:.3f} ms, rotation matrices {r*1e3:.3f} ms "
          f"({B / (d + r):.0f} clips/s host-bound)", flush=True)
    for h, w in ((224, 224), (360, 640), (720, 1280)):
        host = torch.randint(0, 256, (B, T, h, w, 3), generator=g, dtype=torch.uint8).pin_memory()
        dev = host.to("cuda")
        flips, ang = media.draw_augment(n, g)
        k = wall(lambda: media.frame_augment(dev, (224, 224), flips=flips, angles=ang), reps)
        e = wall(lambda: prepare_video(host, "cuda", augment=True, generator=g), reps)
        mb = host.numel() / 1e6
        print(f"frames {h}x{w}: kernel (resident, matrices included) {k*1e3:.2f} ms = {B / k:.0f} clips/s; "
              f"prepare_video from pinned host ({mb:.0f} MB H2D) {e*1e3:.2f} ms = {B / e:.0f} clips/s", flush=True)
    grey = torch.randint(0, 256, (B, 224, 224), generator=g, dtype=torch.uint8).pin_memory()
    m = wall(lambda: prepare_mel(grey, "cuda", augment=True, generator=g), reps)
    print(f"mel slot (grey 224x224, augment) {m*1e3:.2f} ms = {B / m:.0f} clips/s", flush=True)


if __name__ == "__main__":
    main()
