import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from deepfake_amd.models import set_compute_dtype
from deepfake_amd.models.fused import CONFIGS
from deepfake_amd.models.video_swin_transformer import SwinTransformer3D
from deepfake_amd.params import ParamStore
from deepfake_amd import functional as Fn
kw = dict(CONFIGS["c1"]["vst"], drop_path_rate=0.2, use_checkpoint=True)
b = set_compute_dtype(SwinTransformer3D(**kw), torch.bfloat16).cuda().train()
st = ParamStore(b, torch.bfloat16)
names = {id(p): n for n, p in b.named_parameters()}
orig = Fn.grad_use
log = []
def gu(ctx, idx, p):
    if Fn._store(p) is not None and ctx.needs_input_grad[idx]:
        log.append((names.get(id(p)), Fn._RECOMPUTING[0]))
    return orig(ctx, idx, p)
Fn.grad_use = gu
x = torch.randn(2, 8, 3, 112, 112, device="cuda")
y = b.forward_tokens(x, layout="btchw").float().sum()
print("after fwd uses", len(st.uses))
y.backward()
torch.cuda.synchronize()
print("left", [(names[k], v) for k, v in st.uses.items()][:10])
import collections
c = collections.Counter(log)
print([kv for kv in c.items() if "blocks.0" in (kv[0][0] or "")][:12])
# second pass: count grad_ready per name
st.zero_grad()
calls = collections.Counter()
orig_ready = st.grad_ready
def gr(p):
    calls[names.get(id(p))] += 1
    return orig_ready(p)
st.grad_ready = gr
y = b.forward_tokens(x, layout="btchw").float().sum()
y.backward()
torch.cuda.synchronize()
print("ready calls blocks.0:", {k: v for k, v in calls.items() if k and "layers.0.blocks.0" in k})
print("ready calls blocks.1:", {k: v for k, v in calls.items() if k and "layers.0.blocks.1" in k})
print("left2", len(st.uses), sorted(set(names[k].split('.norm')[0].split('.attn')[0].split('.mlp')[0] for k in st.uses)))
