"""Do independent streams overlap on this box, eagerly and inside one captured HIP graph?
Two chains of small-M GEMMs (the wav2vec2 / SwinV2-stage-3 shapes: a few hundred workgroups each),
timed alone, on two streams eagerly, and as one graph with a fork/join."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepfake_amd import kernels as K  # noqa: E402

dt = torch.bfloat16
M, N, Kd = 1568, 2048, 512
xs = [torch.randn(M, Kd, device="cuda").to(dt) for _ in range(2)]
ws = [(torch.randn(N, Kd, device="cuda") * 0.05).to(dt) for _ in range(2)]
outs = [torch.empty(M, N, device="cuda", dtype=dt) for _ in range(2)]
REP = 40


def chain(i):
    for _ in range(REP):
        K.linear(xs[i], ws[i], out=outs[i])


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def two_streams():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        chain(0)
    with torch.cuda.stream(s2):
        chain(1)
    cur.wait_stream(s1)
    cur.wait_stream(s2)


print(f"one chain eager      {timeit(lambda: chain(0)):.3f} ms")
print(f"two chains, 1 stream {timeit(lambda: (chain(0), chain(1))):.3f} ms")
print(f"two chains, 2 streams eager {timeit(two_streams):.3f} ms")
g = torch.cuda.CUDAGraph()
cs = torch.cuda.Stream()
cs.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(cs):
    with torch.cuda.graph(g, stream=cs):
        two_streams()
torch.cuda.current_stream().wait_stream(cs)
print(f"two chains, 2 streams graph {timeit(g.replay):.3f} ms")
g1 = torch.cuda.CUDAGraph()
with torch.cuda.stream(cs):
    with torch.cuda.graph(g1, stream=cs):
        chain(0)
torch.cuda.current_stream().wait_stream(cs)
print(f"one chain graph {timeit(g1.replay):.3f} ms")
ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
with torch.cuda.stream(cs):
    with torch.cuda.graph(ga, stream=cs):
        chain(0)
    with torch.cuda.graph(gb, stream=cs):
        chain(1)
torch.cuda.current_stream().wait_stream(cs)


def two_graphs():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        ga.replay()
    with torch.cuda.stream(s2):
        gb.replay()
    cur.wait_stream(s1)
    cur.wait_stream(s2)


print(f"two graphs replayed on 2 streams {timeit(two_graphs):.3f} ms")
