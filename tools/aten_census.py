"""Census of the stock-torch (aten) kernels inside one eager C2 training step: every aten op that is not a view
or metadata op, with its shapes and the deepfake_amd frame that issued it — the copyBuffer / fill / elementwise
launches of the captured step (rocprof shows their kernels, not their callers).

    python tools/aten_census.py [config] > census.txt
"""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VIEWS = {"view", "_unsafe_view", "as_strided", "slice", "select", "t", "transpose", "permute", "expand", "unsqueeze",
         "squeeze", "reshape", "detach", "alias", "split", "split_with_sizes", "unbind", "chunk", "narrow",
         "_reshape_alias", "diagonal", "empty", "empty_like", "empty_strided", "new_empty", "new_empty_strided",
         "is_same_size", "lift_fresh", "_local_scalar_dense", "item", "set_", "record_stream", "flatten",
         "view_as", "numel", "sym_size", "size", "stride", "is_nonzero", "_has_compatible_shallow_copy_type"}


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func._schema.name.split("::")[-1]
        if name not in VIEWS:
            shapes = tuple(tuple(a.shape) for a in args if isinstance(a, torch.Tensor))[:3]
            where = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "deepfake_amd" in fr.filename or "bench.py" in fr.filename:
                    where = f"{os.path.relpath(fr.filename)}:{fr.lineno}"
                    break
            self.rows[(name, shapes, where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    from bench import synthetic_batch
    from deepfake_amd.ddp import GradBucketer
    from deepfake_amd.models.fused import CONFIGS, build_fused
    from deepfake_amd.optim import FusedSGD
    from deepfake_amd.params import ParamStore
    from deepfake_amd.trainer import TrainStep
    from deepfake_amd import rng
    cfg = CONFIGS[cfg_name]
    torch.manual_seed(1234)
    rng.manual_seed(1234, 0)
    dev = torch.device("cuda", 0)
    model = build_fused(cfg, compute_dtype=torch.bfloat16, regularize=True).to(dev)
    model.train()
    store = ParamStore(model, torch.bfloat16)
    opt = FusedSGD(store, lr=1e-4, momentum=0.9, weight_decay=1e-3)
    step = TrainStep(model, store, opt, GradBucketer(store, bucket_mb=64.0), graph=False)
    feature, label = synthetic_batch(cfg, 8, dev, 1234)
    step(feature, label)
    torch.cuda.synchronize()
    c = Census()
    with c:
        step(feature, label)
    torch.cuda.synchronize()
    tot = sum(c.rows.values())
    print(f"aten ops in one eager step: {tot}")
    for (name, shapes, where), n in sorted(c.rows.items(), key=lambda kv: (-kv[1], kv[0][2])):
        print(f"{n:5d}  {name:28s} {where:45s} {shapes}")


if __name__ == "__main__":
    main()
