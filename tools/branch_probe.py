"""Do the three extractor trunks overlap when their forwards are captured in one HIP graph on three streams?
Times graph replays of each trunk's forward alone and of the fused forward with parallel branches."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synthetic_batch  # noqa: E402
from deepfake_amd.models.fused import CONFIGS, build_fused  # noqa: E402
from deepfake_amd.params import ParamStore  # noqa: E402

cfg = CONFIGS["c2"]
model = build_fused(cfg, compute_dtype=torch.bfloat16, regularize=False).cuda()
model.train()
store = ParamStore(model, torch.bfloat16)
feat, label = synthetic_batch(cfg, 8, torch.device("cuda"), 1)


def cap(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / 5 * 1e3


with torch.no_grad():
    tv = cap(lambda: model.vExtract(feat[0]))
    ta = cap(lambda: model.aExtract(feat[1]))
    tp = cap(lambda: model.paExtract(feat[2]))
    print(f"fwd alone: video {tv:.2f} ms  mel {ta:.2f} ms  wav {tp:.2f} ms  sum {tv + ta + tp:.2f}")
    model.parallel_branches = False
    ts = cap(lambda: model(feat))
    model.parallel_branches = True
    tpar = cap(lambda: model(feat))
    print(f"fused fwd: one stream {ts:.2f} ms  three streams {tpar:.2f} ms")
