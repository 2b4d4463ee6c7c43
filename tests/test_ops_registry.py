"""CPU: the dfk operator library (deepfake_amd/ops.py, torch.library) — schemas, shape propagation through
the fake implementations (what torch.compile / torch.export trace with), and the loud failure on CPU tensors
(no CPU kernel exists)."""
import os

import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import deepfake_amd.ops as O
from deepfake_amd import _lib as L

SCHEMAS = {
    "linear": "dfk::linear(Tensor x, Tensor w, Tensor? b=None) -> Tensor",
    "layer_norm": "dfk::layer_norm(Tensor x, Tensor w, Tensor b, float eps) -> Tensor[]",
    "window_attention": "dfk::window_attention(Tensor qkv, Tensor? rpb, Tensor? pad, SymInt[] dims, SymInt[] window, "
                        "SymInt[] full_window, SymInt[] shift, SymInt heads, SymInt hd, float scale) -> Tensor[]",
}


def test_every_op_registered():
    for name in O.OPS:
        assert hasattr(torch.ops.dfk, name), name
    for name, schema in SCHEMAS.items():
        assert str(getattr(torch.ops.dfk, name).default._schema) == schema


def test_cpu_tensors_fail_loudly():
    x = torch.randn(4, 8)
    w = torch.randn(16, 8)
    with pytest.raises(RuntimeError, match="GPU only"):
        torch.ops.dfk.linear(x, w)
    with pytest.raises(RuntimeError, match="GPU only"):
        torch.ops.dfk.layer_norm(x, torch.ones(8), torch.zeros(8), 1e-5)


def test_fake_shapes():
    bf = torch.bfloat16
    with FakeTensorMode():
        x = torch.empty(100, 96, dtype=bf, device="cuda")
        w = torch.empty(288, 96, dtype=bf, device="cuda")
        assert torch.ops.dfk.linear(x, w).shape == (100, 288)
        dw, db = torch.ops.dfk.linear_dw(torch.empty(100, 288, dtype=bf, device="cuda"), x)
        assert dw.shape == (288, 96) and dw.dtype == torch.float32 and db.shape == (288,)
        y, mean, rstd = torch.ops.dfk.layer_norm(x, torch.empty(96, device="cuda"), torch.empty(96, device="cuda"),
                                                 1e-5)
        assert y.shape == x.shape and mean.shape == (100,) and rstd.dtype == torch.float32
        if not os.path.exists(L.LIB_PATH):
            pytest.skip("libdfk.so not built (run python -m deepfake_amd.build)")
        # Video Swin stage 1 of C2: 8 x 56 x 56 tokens, window 8x7x7 (392 -> 416 padded keys), 3 heads
        qkv = torch.empty(25088, 288, dtype=bf, device="cuda")
        rpb = torch.empty(15 * 13 * 13, 3, device="cuda")
        out, lse, tab = torch.ops.dfk.window_attention(qkv, rpb, None, [1, 8, 56, 56], [8, 7, 7], [8, 7, 7],
                                                       [4, 3, 3], 3, 32, 32 ** -0.5)
        assert out.shape == (25088, 96) and lse.shape == (64 * 3, 416)
        assert tab.numel() == 8 * 3 * 416 * 416 * 2 * 2 // 4   # 8 shift classes x heads x Np^2, bf16, 2 layouts
        _, _, tab0 = torch.ops.dfk.window_attention(qkv, None, None, [1, 8, 56, 56], [8, 7, 7], [8, 7, 7],
                                                    [0, 0, 0], 3, 32, 32 ** -0.5)
        assert tab0.numel() == 0
        img = torch.ops.dfk.mel_image(torch.empty(2, 22050, device="cuda"))
        assert img.shape == (2, 224, 224) and img.dtype == torch.uint8
        fr = torch.ops.dfk.frame_augment(torch.empty(2, 5, 360, 640, 3, dtype=torch.uint8, device="cuda"), None, None)
        assert fr.shape == (2, 5, 3, 224, 224) and fr.dtype == torch.float32
