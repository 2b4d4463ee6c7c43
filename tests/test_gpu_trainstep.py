"""The training runtime's step (deepfake_amd.trainer.TrainStep: flat ParamStore in direct-gradient mode,
fused SGD, the three extractors on parallel HIP streams, optional whole-step HIP-graph capture) gives
the same parameters as the plain sequential eager step, at C1 shapes in fp32 parity mode.
(src/trainer.py:280-297: forward, BCE, backward, SGD(momentum 0.9, weight decay), zero_grad.)"""
import pytest
import torch

import golden_cases as GC
from oracle.fill import named_fill_, synthetic_inputs

pytestmark = pytest.mark.gpu
if torch.cuda.is_available():
    from deepfake_amd.ddp import GradBucketer
    from deepfake_amd.models.fused import build_fused
    from deepfake_amd.optim import FusedSGD
    from deepfake_amd.params import ParamStore
    from deepfake_amd.trainer import TrainStep

DEV = "cuda"


def _run(steps, parallel, graph, dt=torch.float32):
    c = GC.FUSED_C1
    m = named_fill_(build_fused("c1", compute_dtype=dt), c["seed"]).to(DEV)
    m.train()
    store = ParamStore(m, dt)
    step = TrainStep(m, store, FusedSGD(store, 0.01, 0.9, 0.05), GradBucketer(store), graph=graph,
                     parallel_branches=parallel)
    losses = []
    for i in range(steps):
        v, mel, w, lab = synthetic_inputs(c["B"], c["T"], c["H"], c["W"], c["seconds"], seed=c["seed"] + 10 * i)
        loss, _ = step((v.to(DEV), mel.to(DEV), w.to(DEV)), lab.to(DEV))
        losses.append(float(loss))
    torch.cuda.synchronize()
    return store.flat.clone(), losses, m


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max())


def test_parallel_branches_match_sequential():
    ref, lref, m0 = _run(2, parallel=False, graph=False)
    got, lgot, m1 = _run(2, parallel=True, graph=False)
    assert not m0.parallel_branches and m1.parallel_branches
    assert max(abs(a - b) for a, b in zip(lgot, lref)) < 1e-5, (lgot, lref)
    assert _rel(got, ref) < 1e-5


def test_graph_captured_step_matches_eager():
    """Step 1 runs eager and captures the step; steps 2-3 replay the graph on new inputs copied into the
    captured buffers; parameters and losses equal three eager steps."""
    ref, lref, _ = _run(3, parallel=True, graph=False)
    got, lgot, _ = _run(3, parallel=True, graph=True)
    assert max(abs(a - b) for a, b in zip(lgot, lref)) < 1e-5, (lgot, lref)
    assert _rel(got, ref) < 1e-5


def test_captured_overlapped_allreduce_single_rank():
    """The step graph with the bucket all-reduces captured where backward completes each bucket (§8e):
    one RCCL rank on the box's GPU (DFK_DDP_FORCE=1 enables the bucketer at world size 1), C1, eager vs
    graph-replayed steps — the overlapped form (BatchNorm broadcast inside the graph) must be the one captured
    and the parameters must agree.  No sleep: the capture waits until the flight recorder shows the watchdog
    retired the eager replica's fresh RCCL works (deepfake_amd.ddp.watchdog_idle)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DFK_DDP_FORCE="1", TORCH_NCCL_CUDA_EVENT_CACHE="0", TORCH_FR_BUFFER_SIZE="256",
               MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", "29531",
                        os.path.join(root, "tools", "ddp_graph_probe.py"), "c1"],
                       env=env, capture_output=True, text=True, timeout=110, cwd=root)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "captured overlapped all-reduces: True" in out, out[-3000:]
    assert "captured BN broadcast: True" in out, out[-3000:]
    assert "\nok" in out, out[-3000:]


def _run_accum(windows, accum, graph, dt=torch.float32):
    c = GC.FUSED_C1
    m = named_fill_(build_fused("c1", compute_dtype=dt), c["seed"]).to(DEV)
    m.train()
    store = ParamStore(m, dt)
    step = TrainStep(m, store, FusedSGD(store, 0.01, 0.9, 0.05), GradBucketer(store), graph=graph)
    losses = []
    for i in range(windows * accum):
        v, mel, w, lab = synthetic_inputs(c["B"], c["T"], c["H"], c["W"], c["seconds"], seed=c["seed"] + 7 * i)
        loss, _ = step.micro((v.to(DEV), mel.to(DEV), w.to(DEV)), lab.to(DEV), (i + 1) % accum == 0, accum)
        losses.append(float(loss))
    torch.cuda.synchronize()
    return store.flat.clone(), losses, step


def test_graphed_accumulation_matches_eager():
    """--accum_step 4 (the reference default, config.py:31; src/trainer.py:280-297) with graphs: one eager window,
    then the non-final and final micro-step graphs replayed for two more windows — parameters and every
    micro-step's loss equal the all-eager run (C1, fp32 parity mode)."""
    ref, lref, _ = _run_accum(3, 4, graph=False)
    got, lgot, st = _run_accum(3, 4, graph=True)
    assert st.agraphs is not None and st.graph_mode, "accumulation graphs were not captured"
    assert max(abs(a - b) for a, b in zip(lgot, lref)) < 1e-5, (lgot, lref)
    assert _rel(got, ref) < 1e-5
