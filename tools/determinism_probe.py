"""Run-to-run determinism of the fused training step: the same model, weights and inputs, forward + BCE backward
twice (eager, bf16 or fp32); reports which gradient tensors differ between the two runs and by how much.

    python tools/determinism_probe.py [c1|c2] [bf16|fp32] [B]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.fill import named_fill_, synthetic_inputs  # noqa: E402


def main():
    from deepfake_amd.models.fused import CONFIGS, build_fused
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    dt = torch.bfloat16 if (sys.argv[2] if len(sys.argv) > 2 else "bf16") == "bf16" else torch.float32
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    cfg = CONFIGS[cfg_name]
    m = named_fill_(build_fused(cfg_name, compute_dtype=dt), 181).cuda().train()
    video, mel, wave, label = synthetic_inputs(B, cfg["T"], cfg["H"], cfg["W"], cfg["seconds"], seed=182)
    x = (video.cuda(), mel.cuda(), wave.cuda())
    label = label.cuda()
    runs = []
    for _ in range(2):
        for p in m.parameters():
            p.grad = None
        p_ = m(x)
        loss = torch.nn.BCELoss()(p_.float(), label)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((loss.item(), m.last_logits.float().clone(),
                     {n: q.grad.detach().float().clone() for n, q in m.named_parameters() if q.grad is not None}))
    (l0, z0, g0), (l1, z1, g1) = runs
    print(f"loss {l0!r} vs {l1!r} equal={l0 == l1}; logits equal={torch.equal(z0, z1)}")
    diffs = []
    for n in g0:
        d = (g0[n] - g1[n]).abs().max().item()
        if d > 0:
            diffs.append((d / max(g0[n].abs().max().item(), 1e-30), n))
    diffs.sort(reverse=True)
    print(f"{len(diffs)} of {len(g0)} gradient tensors differ between identical runs")
    for r, n in diffs[:40]:
        print(f"  {r:.3e}  {n}")
    num = sum(((g0[n] - g1[n]).double() ** 2).sum().item() for n in g0)
    den = sum((g0[n].double() ** 2).sum().item() for n in g0)
    print(f"relative L2 between the runs: {(num / den) ** 0.5:.3e}")


if __name__ == "__main__":
    main()
