"""GPU: the dfk operator library (torch.ops.dfk.*, deepfake_amd/ops.py) against torch fp32 references,
through autograd, torch.library.opcheck and torch.compile (aot_eager: the registered fake + autograd
implementations trace; no Triton codegen)."""
import pytest
import torch
import torch.nn.functional as F

from tests.test_gpu_wattn import ref_attention

pytestmark = pytest.mark.gpu
DEV = "cuda"
if torch.cuda.is_available():
    import deepfake_amd.ops  # noqa: F401  (registers torch.ops.dfk)


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_linear_autograd(dt):
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(777, 384, device=DEV, generator=g).to(dt).requires_grad_(True)
    w = (0.05 * torch.randn(1536, 384, device=DEV, generator=g)).to(dt).requires_grad_(True)
    b = torch.randn(1536, device=DEV, generator=g).to(dt).requires_grad_(True)
    y = torch.ops.dfk.linear(x, w, b)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = F.linear(xr, wr, br)
    yr.backward(dy.float())
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    for got, ref, name in ((y, yr, "y"), (x.grad, xr.grad, "dx"), (w.grad, wr.grad, "dw"), (b.grad, br.grad, "db")):
        assert got.dtype == dt and _rel(got, ref) < tol, (name, _rel(got, ref))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layer_norm_autograd(dt):
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.randn(1000, 192, device=DEV, generator=g).to(dt).requires_grad_(True)
    w = (1 + 0.1 * torch.randn(192, device=DEV, generator=g)).to(dt).requires_grad_(True)
    b = (0.1 * torch.randn(192, device=DEV, generator=g)).to(dt).requires_grad_(True)
    y = torch.ops.dfk.layer_norm(x, w, b, 1e-5)[0]
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = F.layer_norm(xr, (192,), wr, br, 1e-5)
    yr.backward(dy.float())
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    for got, ref, name in ((y, yr, "y"), (x.grad, xr.grad, "dx"), (w.grad, wr.grad, "dw"), (b.grad, br.grad, "db")):
        assert _rel(got, ref) < tol, (name, _rel(got, ref))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shift", [(0, 0, 0), (2, 3, 3)])
def test_window_attention_autograd(dt, shift):
    dims, window, fw, heads, hd = (1, 4, 10, 10), (4, 7, 7), (4, 7, 7), 2, 32
    g = torch.Generator(device=DEV).manual_seed(5)
    C = heads * hd
    rows = 400
    qkv = torch.randn(rows, 3 * C, device=DEV, generator=g).to(dt).requires_grad_(True)
    pad = (0.3 * torch.randn(3 * C, device=DEV, generator=g)).to(dt).requires_grad_(True)
    rpb = (0.5 * torch.randn(7 * 13 * 13, heads, device=DEV, generator=g)).requires_grad_(True)
    out = torch.ops.dfk.window_attention(qkv, rpb, pad, list(dims), list(window), list(fw), list(shift), heads, hd,
                                         hd ** -0.5)[0]
    dout = torch.randn_like(out)
    out.backward(dout)
    qr, pr, rr = (t.detach().float().requires_grad_(True) for t in (qkv, pad, rpb))
    ref = ref_attention(qr, [pr[:C], pr[C:2 * C], pr[2 * C:]], dims, window, fw, shift, heads, hd, hd ** -0.5, rr)
    ref.backward(dout.float())
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    for got, r, name in ((out, ref, "out"), (qkv.grad, qr.grad, "dqkv"), (rpb.grad, rr.grad, "drpb"),
                         (pad.grad, pr.grad, "dpad")):
        assert _rel(got, r) < tol, (name, _rel(got, r))


def test_opcheck():
    """Schema / fake-tensor / autograd-registration checks of torch.library on real GPU calls."""
    utils = ("test_schema", "test_autograd_registration", "test_faketensor")
    x = torch.randn(64, 96, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(128, 96, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    torch.library.opcheck(torch.ops.dfk.linear, (x, w, None), test_utils=utils)
    torch.library.opcheck(torch.ops.dfk.layer_norm, (x, torch.ones(96, device=DEV, dtype=torch.bfloat16),
                                                     torch.zeros(96, device=DEV, dtype=torch.bfloat16), 1e-5),
                          test_utils=utils)
    qkv = torch.randn(400, 192, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    rpb = torch.randn(7 * 13 * 13, 2, device=DEV, requires_grad=True)
    torch.library.opcheck(torch.ops.dfk.window_attention,
                          (qkv, rpb, None, [1, 4, 10, 10], [4, 7, 7], [4, 7, 7], [2, 3, 3], 2, 32, 32 ** -0.5),
                          test_utils=utils)


def test_torch_compile_block():
    """A pre-norm attention block written with torch.ops.dfk traces under torch.compile (fullgraph) and agrees
    with the eager call."""
    dims, window, heads, hd = [1, 4, 14, 14], [4, 7, 7], 2, 32
    C = heads * hd
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(784, C, device=DEV, generator=g, dtype=torch.bfloat16, requires_grad=True)
    lw, lb = torch.ones(C, device=DEV, dtype=torch.bfloat16), torch.zeros(C, device=DEV, dtype=torch.bfloat16)
    wq = (0.1 * torch.randn(3 * C, C, device=DEV, generator=g)).to(torch.bfloat16).requires_grad_(True)
    rpb = (0.5 * torch.randn(7 * 13 * 13, heads, device=DEV, generator=g)).requires_grad_(True)

    def block(x, wq, rpb):
        h = torch.ops.dfk.layer_norm(x, lw, lb, 1e-5)[0]
        qkv = torch.ops.dfk.linear(h, wq, None)
        o = torch.ops.dfk.window_attention(qkv, rpb, None, dims, window, window, [2, 3, 3], heads, hd, hd ** -0.5)[0]
        return x + o

    y0 = block(x, wq, rpb)
    y0.float().square().sum().backward()
    ref = [t.grad.clone() for t in (x, wq, rpb)]
    for t in (x, wq, rpb):
        t.grad = None
    y1 = torch.compile(block, backend="aot_eager", fullgraph=True)(x, wq, rpb)
    y1.float().square().sum().backward()
    assert _rel(y1, y0) < 1e-2
    for t, r in zip((x, wq, rpb), ref):
        assert _rel(t.grad, r) < 2e-2
