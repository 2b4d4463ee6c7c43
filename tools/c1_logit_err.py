"""C1 bf16 training step: the SwinV2 logit_scale gradient norms against the reference's fp32 step and the
reference's own bf16 error (tests/golden/fused_c1.npz gn:*, fused_c1_grads.npz ea:*), plus the worst tensor
overall.  A/B: DFK_COS_DSCORE=0 (q-hat . dq' in the cosine backward), DFK_WATTN_V6MIN (v6 from that many
query blocks; 2 puts the 49-token SwinV2 windows on v6)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import golden_cases as GC  # noqa: E402
from fixtures import keys, load  # noqa: E402
from oracle.fill import named_fill_, synthetic_inputs  # noqa: E402
from deepfake_amd.models.fused import build_fused  # noqa: E402

c = GC.FUSED_C1
fx, ea = load(c["name"]), load("fused_c1_grads")
m = named_fill_(build_fused("c1", compute_dtype=torch.bfloat16), c["seed"]).cuda()
video, mel, wave, label = synthetic_inputs(c["B"], c["T"], c["H"], c["W"], c["seconds"], seed=c["seed"] + 1)
m.train()
p = m((video.cuda(), mel.cuda(), wave.cuda()))
torch.nn.BCELoss()(p.float(), label.cuda()).backward()
names = dict(m.named_parameters())
tag = f"dscore={os.environ.get('DFK_COS_DSCORE', '1')} v6min={os.environ.get('DFK_WATTN_V6MIN', '4')}"
worst = (None, 0.0, 0.0)
for k in keys(fx, "gn:"):
    n = k[3:]
    ref, got = float(fx[k]), float(names[n].grad.norm())
    e = float(ea.get("ea:" + n, 0.0))
    r = abs(got - ref) / max(ref, 1e-12)
    if "logit_scale" in n:
        print(f"{tag} {n}: rel {r:.4f}  ref-bf16 {e:.4f}  ratio {r / max(e, 1e-9):.2f}")
    if ref > 1e-4 and r / max(2e-2, 6 * e) > worst[2]:
        worst = (n, r, r / max(2e-2, 6 * e))
print(f"{tag} worst tensor vs its gate: {worst}")
