"""Debug: dfk Swin3D block vs oracle block gradients (fp32 and bf16), golden seeds and others."""
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests", "golden"))
import oracle.vst as OV  # noqa: E402
from oracle.fill import named_fill_, randn  # noqa: E402
import deepfake_amd.models.video_swin_transformer as V  # noqa: E402


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).abs().max() / b.abs().max()).item()


for dt in (torch.float32, torch.bfloat16):
    for (shape, seed) in [((1, 16, 14, 14), 5), ((1, 16, 14, 14), 21), ((2, 8, 14, 14), 5)]:
        B, D, H, W = shape
        blk = named_fill_(V.SwinTransformerBlock3D(96, 3, window_size=(8, 7, 7), shift_size=(4, 3, 3)), seed).cuda()
        ob = named_fill_(OV.SwinTransformerBlock3D(96, 3, (8, 7, 7), (4, 3, 3)), seed)
        x = randn(seed + 1, (B, D, H, W, 96)).cuda()
        xb = x.to(dt).requires_grad_(True)
        y = blk(xb, None)
        xf = xb.detach().float().cpu().requires_grad_(True)
        ref = ob(xf)
        dy = randn(seed + 2, y.shape).cuda().to(dt)
        y.backward(dy)
        ref.backward(dy.float().cpu())
        ours = dict(blk.named_parameters())
        print(dt, shape, seed, "y %.2e dx %.2e" % (rel(y, ref), rel(xb.grad, xf.grad)),
              " ".join("%s %.2e" % (n.split(".")[-2] + "." + n.split(".")[-1], rel(ours[n].grad, p.grad))
                       for n, p in ob.named_parameters()), flush=True)
        print("   |dy| %.3f  fc2.bias ours %s ref %s" % (dy.float().abs().max().item(),
              ours["mlp.fc2.bias"].grad[:3].tolist(), ob.mlp.fc2.bias.grad[:3].tolist()), flush=True)
