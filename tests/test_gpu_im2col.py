"""GPU: patch im2col (Conv3d / Conv2d with kernel == stride; PatchEmbed3D video_swin_transformer.py:436-453,
SwinV2 PatchEmbed swin_transformer2d.py:461-477) vs a torch fp32 restatement, on the row-staged vector
kernel (aligned fp32 rows) and the element-wise kernel (anything else), with zero padding of T / H / W."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if torch.cuda.is_available():
    from deepfake_amd import kernels as K

DEV = "cuda"


def ref_cols(x, layout, patch):
    """cols[(b, d, h, w)][(c, kd, kh, kw)] of the zero-padded clip / image."""
    if layout == "bchw":
        x = x.unsqueeze(2)   # [B, C, 1, H, W]
        pd, ph, pw = 1, patch[0], patch[1]
    else:
        if layout == "btchw":
            x = x.permute(0, 2, 1, 3, 4)
        pd, ph, pw = patch
    B, C, T, H, W = x.shape
    Do, Ho, Wo = -(-T // pd), -(-H // ph), -(-W // pw)
    xp = torch.zeros(B, C, Do * pd, Ho * ph, Wo * pw, device=x.device)
    xp[:, :, :T, :H, :W] = x.float()
    v = xp.view(B, C, Do, pd, Ho, ph, Wo, pw).permute(0, 2, 4, 6, 1, 3, 5, 7)
    return v.reshape(B * Do * Ho * Wo, C * pd * ph * pw)


CASES = [
    ((2, 8, 3, 32, 32), "btchw", (2, 4, 4)),     # aligned rows: row-staged kernel
    ((1, 5, 3, 18, 24), "btchw", (2, 4, 4)),     # T and H padded
    ((1, 3, 3, 16, 28), "btchw", (1, 4, 8)),     # W padded inside a staged row (tail quad)
    ((1, 3, 4, 19, 22), "bcthw", (2, 4, 4)),     # rows not 16-B aligned: element-wise kernel
    ((2, 3, 64, 64), "bchw", (4, 4)),            # SwinV2 mel PatchEmbed
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape,layout,patch", CASES, ids=[str(i) for i in range(len(CASES))])
def test_patch_im2col(shape, layout, patch, dt):
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.randn(*shape, device=DEV, generator=g)
    cols, grid = K.patch_im2col(x, layout, patch, dt)
    ref = ref_cols(x, layout, patch)
    assert cols.shape == ref.shape
    assert grid[0] * grid[1] * grid[2] * grid[3] == ref.shape[0]
    # a pure gather: exact in fp32, one rounding in bf16
    torch.testing.assert_close(cols.float(), ref.to(dt).float(), rtol=0, atol=0)
