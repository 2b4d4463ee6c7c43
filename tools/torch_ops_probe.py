"""Which stock PyTorch ops run inside the C2 training step (fills, copies, where, adds), with their Python call
sites: one eager warm-up step, then one profiled eager step (torch.profiler, stacks).

    python tools/torch_ops_probe.py [config] [batch]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from deepfake_amd import rng  # noqa: E402
from deepfake_amd.ddp import GradBucketer  # noqa: E402
from deepfake_amd.models.fused import CONFIGS, build_fused  # noqa: E402
from deepfake_amd.optim import FusedSGD  # noqa: E402
from deepfake_amd.params import ParamStore  # noqa: E402
from deepfake_amd.trainer import TrainStep  # noqa: E402

WATCH = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::where", "aten::add", "aten::add_", "aten::clone",
         "aten::cat", "aten::to", "aten::_to_copy", "aten::mul", "aten::zeros", "aten::zeros_like", "aten::contiguous")


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    cfg = CONFIGS[name]
    torch.manual_seed(1234)
    rng.manual_seed(1234, 0)
    model = build_fused(cfg, compute_dtype=torch.bfloat16, regularize=True).cuda()
    model.train()
    store = ParamStore(model, torch.bfloat16)
    opt = FusedSGD(store, lr=1e-4, momentum=0.9, weight_decay=1e-3)
    step = TrainStep(model, store, opt, GradBucketer(store, bucket_mb=64.0), graph=False)
    feature, label = bench.synthetic_batch(cfg, B, torch.device("cuda"), 1234)
    step(feature, label)
    torch.cuda.synchronize()
    import collections
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    seen = collections.Counter()

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func.overloadpacket.__name__)
            if any(w in name for w in ("fill", "zero", "copy", "where", "add", "clone", "cat", "to_copy", "mul")):
                fr = [f for f in traceback.extract_stack()[:-1] if "deepfake_amd" in f.filename]
                site = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-3:][::-1])
                seen[(name, site)] += 1
            return func(*args, **(kwargs or {}))

    with Log():
        step(feature, label)
    torch.cuda.synchronize()
    for (name, site), n in seen.most_common(45):
        print(f"{n:4d}x {name:18s} {site}")

if __name__ == "__main__":
    main()
