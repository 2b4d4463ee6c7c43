"""Video Swin Transformer 3D on MI355X — drop-in for
/root/reference/src/models/video_swin_transformer.py (classes, constructor
signatures, forward layouts and state_dict keys kept).

Hot path layout: channels-last token rows [B, D, H, W, C] (the layout the
reference's blocks already use), so LayerNorm, qkv/proj/MLP GEMMs and the
window attention read one token-major buffer; cyclic shift, padding and
window partition/reverse are index arithmetic inside dfk_wattn_* — no
roll/permute copies.  Stage boundaries ([B,C,D,H,W] in the reference's
BasicLayer/SwinTransformer3D API) are converted only at the public API
entry/exit; the fused model's video extractor (VSTFeat) never leaves the
token layout.

Stochastic depth (timm DropPath, :214) runs in training mode as a per-clip
mask fused into the proj / fc2 GEMM epilogues (rng.Drop mode 2, one draw per
clip's tokens, scaled 1/(1-p)); the backward applies the same mask to the
branch gradient.  Plain dropout / attention dropout with p > 0 (drop_rate,
attn_drop_rate: 0 in every reference configuration) raise.
"""
from functools import lru_cache

import torch
import torch.nn as nn

from .. import functional as Fn
from .. import rng
from ..utils import Mlp


def window_partition(x, window_size):
    """video_swin_transformer.py:42-54 (API utility; the hot path never materialises windows)."""
    B, D, H, W, C = x.shape
    wd, wh, ww = window_size
    x = x.view(B, D // wd, wd, H // wh, wh, W // ww, ww, C)
    return x.permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(-1, wd * wh * ww, C)


def window_reverse(windows, window_size, B, D, H, W):
    """video_swin_transformer.py:57-70."""
    wd, wh, ww = window_size
    x = windows.view(B, D // wd, H // wh, W // ww, wd, wh, ww, -1)
    return x.permute(0, 1, 4, 2, 5, 3, 6, 7).reshape(B, D, H, W, -1)


def get_window_size(x_size, window_size, shift_size=None):
    """video_swin_transformer.py:75-88 (Q6): a dim no larger than the window is
    one window and is never shifted."""
    ws = tuple(min(s, w) if s <= w else w for s, w in zip(x_size, window_size))
    if shift_size is None:
        return ws
    ss = tuple(0 if s <= w else sh for s, w, sh in zip(x_size, window_size, shift_size))
    return ws, ss


def _region(P, w, s, device):
    i = torch.arange(P, device=device)
    if s == 0:
        return torch.full((P,), 2, device=device, dtype=torch.long)
    return torch.where(i < P - w, 0, torch.where(i < P - s, 1, 2))


@lru_cache()
def compute_mask(D, H, W, window_size, shift_size, device):
    """video_swin_transformer.py:319-333: [nW, N, N] with 0 / -100.0 (Q4).
    (The hot path derives the same mask from region labels inside the kernel.)"""
    lab = (_region(D, window_size[0], shift_size[0], device)[:, None, None] * 9
           + _region(H, window_size[1], shift_size[1], device)[None, :, None] * 3
           + _region(W, window_size[2], shift_size[2], device)[None, None, :])
    mw = window_partition(lab[None, ..., None].float(), window_size).squeeze(-1)
    diff = mw.unsqueeze(1) - mw.unsqueeze(2)
    return torch.where(diff != 0, -100.0, 0.0)


def _rel_index(window_size):
    Wd, Wh, Ww = window_size
    t = torch.arange(Wd * Wh * Ww)
    d, h, w = t // (Wh * Ww), (t // Ww) % Wh, t % Ww
    return (((d[:, None] - d[None, :] + Wd - 1) * (2 * Wh - 1) + (h[:, None] - h[None, :] + Wh - 1)) * (2 * Ww - 1)
            + (w[:, None] - w[None, :] + Ww - 1))


class WindowAttention3D(nn.Module):
    """video_swin_transformer.py:91-173.  forward(x [B_,N,C] windows, mask [nW,N,N] or None)."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=False, qk_scale=None, attn_drop=0., proj_drop=0.):
        super().__init__()
        self.dim, self.window_size, self.num_heads = dim, tuple(window_size), num_heads
        # attn_drop (:165, on the softmax probabilities: the attention kernels' DROP variants) and proj_drop
        # (:171, the proj GEMM epilogue) as device dropout sites, created only when p > 0
        self.attn_drop = rng.Drop(attn_drop) if attn_drop > 0 else None
        self.proj_drop = rng.Drop(proj_drop) if proj_drop > 0 else None
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        L = (2 * window_size[0] - 1) * (2 * window_size[1] - 1) * (2 * window_size[2] - 1)
        self.relative_position_bias_table = nn.Parameter(torch.zeros(L, num_heads))
        self.register_buffer("relative_position_index", _rel_index(self.window_size))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=.02)

    def drop_specs(self):
        """(attention-probability, proj-output) dropout specs; None outside training or at p = 0."""
        on = lambda d: d.spec() if d is not None and self.training else None   # noqa: E731
        return on(self.attn_drop), on(self.proj_drop)

    def core(self, qkv, dims, window, shift, mask=None):
        """Attention core over a token-major qkv buffer; returns [rows, C] (pre-proj).  Attention dropout
        (training, attn_drop > 0) masks P in the kernel: unit (window, head) row q col k of the mask stream."""
        hd = self.dim // self.num_heads
        geo = (tuple(dims), tuple(window), self.window_size, tuple(shift), self.num_heads, hd, self.scale)
        padded = any(n % w for n, w in zip(dims[1:], window))
        return Fn.window_attention(qkv, self.relative_position_bias_table,
                                   self.qkv.bias if padded else None, geo, mask, drop=self.drop_specs()[0])

    def forward(self, x, mask=None):
        B_, N, C = x.shape
        qkv = Fn.linear(x.reshape(-1, C), self.qkv.weight, self.qkv.bias)
        m = mask.float().contiguous() if mask is not None else None
        o = self.core(qkv, (B_, 1, 1, N), (1, 1, N), (0, 0, 0), mask=m)
        return Fn.linear(o, self.proj.weight, self.proj.bias, drop=self.drop_specs()[1]).view(B_, N, C)


class SwinTransformerBlock3D(nn.Module):
    """video_swin_transformer.py:176-278; forward(x [B,D,H,W,C], mask_matrix).
    The shift mask is recomputed arithmetically in the kernel (mask_matrix is
    accepted for API compatibility and equals compute_mask's output)."""

    def __init__(self, dim, num_heads, window_size=(2, 7, 7), shift_size=(0, 0, 0), mlp_ratio=4., qkv_bias=True,
                 qk_scale=None, drop=0., attn_drop=0., drop_path=0., act_layer=nn.GELU, norm_layer=nn.LayerNorm,
                 use_checkpoint=False):
        super().__init__()
        self.dim, self.num_heads = dim, num_heads
        self.window_size, self.shift_size = tuple(window_size), tuple(shift_size)
        self.mlp_ratio, self.use_checkpoint = mlp_ratio, use_checkpoint
        assert all(0 <= s < w for s, w in zip(self.shift_size, self.window_size)), "shift_size must in 0-window_size"
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention3D(dim, window_size=self.window_size, num_heads=num_heads, qkv_bias=qkv_bias,
                                      qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)
        self.drop_path = nn.Identity()
        # timm DropPath is called once per branch: two independent per-sample draws
        self.dp = (rng.Drop(drop_path, mode=2), rng.Drop(drop_path, mode=2)) if drop_path > 0 else None
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)
        self.mx = False   # MX-fp8 qkv / proj / fc1 / fc2 GEMMs (models.set_fp8; C4's fp8 path)

    def _part1(self, xn, dims):
        """qkv -> shifted-window attention (pad/roll/partition in-kernel) of LN1's output; pre-proj rows."""
        B, D, H, W = dims
        C = xn.shape[-1]
        ws, ss = get_window_size((D, H, W), self.window_size, self.shift_size)
        qkv = Fn.linear(xn.reshape(-1, C), self.attn.qkv.weight, self.attn.qkv.bias, mx=self.mx)
        return self.attn.core(qkv, (B, D, H, W), ws, ss)

    def forward_part1(self, x, mask_matrix=None):
        """LN1 -> qkv -> shifted-window attention; returns pre-proj rows."""
        return self._part1(Fn.layer_norm(x, self.norm1), x.shape[:4])

    def _attn_branch(self, x, dp):
        """x + DropPath(proj_drop(proj(W-MSA(LN1 x))))  (forward_part1 + the first residual, :266-271).  The
        residual reads LN1's skip alias of x, so x's two gradients meet inside the LN backward.  One dropout
        runs in the proj epilogue; with both proj_drop and DropPath active the DropPath is a separate pass."""
        B, D, H, W, C = x.shape
        xn, xs = Fn.layer_norm(x, self.norm1, skip=True)
        o = self._part1(xn, (B, D, H, W))
        pd = self.attn.drop_specs()[1]
        if pd is not None and dp is not None:
            z = Fn.linear(o, self.attn.proj.weight, self.attn.proj.bias, drop=pd, mx=self.mx)
            return (xs.reshape(-1, C) + Fn.DropoutFn.apply(z, dp)).view(B, D, H, W, C)
        return Fn.linear(o, self.attn.proj.weight, self.attn.proj.bias, residual=xs.reshape(-1, C),
                         drop=dp if pd is None else pd, mx=self.mx).view(B, D, H, W, C)

    def _mlp_branch(self, x, dp):
        """x + DropPath(mlp(LN2 x))  (forward_part2 + the second residual, :273-276); Mlp's two dropouts
        (after the GELU, after fc2) in the fc1 / fc2 epilogues."""
        xn, xs = Fn.layer_norm(x, self.norm2, skip=True)
        da, do = self.mlp.drop_specs()
        if do is not None and dp is not None:
            m = Fn.mlp(xn, self.mlp.fc1, self.mlp.fc2, drop_act=da, drop_out=do, mx=self.mx)
            return xs + Fn.DropoutFn.apply(m.reshape(-1, xs.shape[-1]), dp).view(xs.shape)
        return Fn.mlp(xn, self.mlp.fc1, self.mlp.fc2, residual=xs, drop_act=da, drop_out=dp if do is None else do,
                      mx=self.mx)

    def forward(self, x, mask_matrix=None):
        B, D, H, W, C = x.shape
        on = self.dp is not None and self.training
        dp = (self.dp[0].spec(D * H * W), self.dp[1].spec(D * H * W)) if on else (None, None)
        if self.use_checkpoint and self.training and torch.is_grad_enabled():   # :267-276
            x = Fn.checkpoint(self._attn_branch, x, dp[0])
            x = Fn.checkpoint(self._mlp_branch, x, dp[1])
        else:
            x = self._mlp_branch(self._attn_branch(x, dp[0]), dp[1])
        return x.view(B, D, H, W, C)


class PatchMerging(nn.Module):
    """video_swin_transformer.py:281-316: 2x2 gather (Q7 order), LN(4C), Linear(4C->2C, no bias)."""

    def __init__(self, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = norm_layer(4 * dim)

    def forward(self, x):
        B, D, H, W, C = x.shape
        m = Fn.PatchMergeFn.apply(x.reshape(-1, C).contiguous(), (B, D, H, W))
        y = Fn.linear(Fn.layer_norm(m, self.norm), self.reduction.weight)
        return y.view(B, D, (H + 1) // 2, (W + 1) // 2, 2 * C)


class BasicLayer(nn.Module):
    """video_swin_transformer.py:336-417; forward(x [B,C,D,H,W]) -> [B,C',D,H',W']."""

    def __init__(self, dim, depth, num_heads, window_size=(1, 7, 7), mlp_ratio=4., qkv_bias=False, qk_scale=None,
                 drop=0., attn_drop=0., drop_path=0., norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False):
        super().__init__()
        self.window_size = tuple(window_size)
        self.shift_size = tuple(i // 2 for i in window_size)
        self.depth, self.use_checkpoint = depth, use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock3D(dim=dim, num_heads=num_heads, window_size=window_size,
                                   shift_size=(0, 0, 0) if (i % 2 == 0) else self.shift_size, mlp_ratio=mlp_ratio,
                                   qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop, attn_drop=attn_drop,
                                   drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                   norm_layer=norm_layer, use_checkpoint=use_checkpoint)
            for i in range(depth)])
        self.downsample = downsample(dim=dim, norm_layer=norm_layer) if downsample is not None else None

    def forward_tokens(self, x):
        """channels-last [B,D,H,W,C] in and out (the hot path)."""
        for blk in self.blocks:
            x = blk(x)
        if self.downsample is not None:
            x = self.downsample(x)
        return x

    def forward(self, x):
        x = self.forward_tokens(x.permute(0, 2, 3, 4, 1).contiguous())
        return x.permute(0, 4, 1, 2, 3).contiguous()


class PatchEmbed3D(nn.Module):
    """video_swin_transformer.py:420-460: Conv3d(kernel=stride=patch) as im2col +
    MFMA GEMM, then LayerNorm; padding of T/H/W to the patch grid is implicit."""

    def __init__(self, patch_size=(2, 4, 4), in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        self.patch_size, self.in_chans, self.embed_dim = tuple(patch_size), in_chans, embed_dim
        self.proj = nn.Conv3d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None
        self.compute_dtype = torch.float32

    def fused_ok(self, x):
        """The fused bf16 kernel's geometry: 3 input channels, 2x4x4 patches, C in {96, 128}, LayerNorm,
        an fp32 clip whose W stride is 1, <= 256 pixels per row (fp32 parity mode keeps the 3-pass path)."""
        return (self.compute_dtype == torch.bfloat16 and self.norm is not None and self.in_chans == 3 and
                self.patch_size == (2, 4, 4) and self.embed_dim in (96, 128) and x.dtype == torch.float32 and
                x.stride(-1) == 1 and all(s % 4 == 0 for s in x.stride()[:-1]) and x.shape[-1] <= 256 and
                x.shape[-1] % 4 == 0 and
                x.data_ptr() % 16 == 0 and not getattr(self, "force_unfused", False))

    def tokens(self, x, layout="bcthw"):
        """-> channels-last [B, D', H', W', C] in the compute dtype."""
        if layout == "btchw":
            B, T, _, H, W = x.shape
        else:
            B, _, T, H, W = x.shape
        pd, ph, pw = self.patch_size
        Do, Ho, Wo = -(-T // pd), -(-H // ph), -(-W // pw)
        if self.fused_ok(x):   # one pass: pad + Conv3d + LayerNorm (dfk_patch_embed_fwd)
            y = Fn.PatchEmbedLNFn.apply(x, self.proj.weight, self.proj.bias, self.norm.weight, self.norm.bias, layout,
                                        self.norm.eps)
            return y.view(B, Do, Ho, Wo, self.embed_dim)
        y = Fn.PatchEmbedFn.apply(x, self.proj.weight, self.proj.bias, layout, self.patch_size, self.compute_dtype)
        if self.norm is not None:
            y = Fn.layer_norm(y, self.norm)
        return y.view(B, Do, Ho, Wo, self.embed_dim)

    def forward(self, x):
        return self.tokens(x).permute(0, 4, 1, 2, 3).contiguous()


class SwinTransformer3D(nn.Module):
    """video_swin_transformer.py:462-686; forward(x [B,C,T,H,W]) -> [B,8C,T',H',W']."""

    def __init__(self, pretrained=None, pretrained2d=True, patch_size=(4, 4, 4), in_chans=3, embed_dim=96,
                 depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24], window_size=(2, 7, 7), mlp_ratio=4., qkv_bias=True,
                 qk_scale=None, drop_rate=0., attn_drop_rate=0., drop_path_rate=0.2, norm_layer=nn.LayerNorm,
                 patch_norm=False, frozen_stages=-1, use_checkpoint=False):
        super().__init__()
        self.pretrained, self.pretrained2d = pretrained, pretrained2d
        self.num_layers, self.embed_dim = len(depths), embed_dim
        self.patch_norm, self.frozen_stages = patch_norm, frozen_stages
        self.window_size, self.patch_size = tuple(window_size), tuple(patch_size)
        self.patch_embed = PatchEmbed3D(patch_size=patch_size, in_chans=in_chans, embed_dim=embed_dim,
                                        norm_layer=norm_layer if patch_norm else None)
        self.pos_drop = nn.Identity() if drop_rate == 0 else nn.Dropout(p=drop_rate)
        dpr = [float(x) for x in torch.linspace(0, drop_path_rate, sum(depths))]
        self.layers = nn.ModuleList()
        for i in range(self.num_layers):
            self.layers.append(BasicLayer(
                dim=int(embed_dim * 2 ** i), depth=depths[i], num_heads=num_heads[i], window_size=window_size,
                mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop_rate, attn_drop=attn_drop_rate,
                drop_path=dpr[sum(depths[:i]):sum(depths[:i + 1])], norm_layer=norm_layer,
                downsample=PatchMerging if i < self.num_layers - 1 else None, use_checkpoint=use_checkpoint))
        self.num_features = int(embed_dim * 2 ** (self.num_layers - 1))
        self.norm = norm_layer(self.num_features)
        self._freeze_stages()

    def _freeze_stages(self):
        if self.frozen_stages >= 0:
            for p in self.patch_embed.parameters():
                p.requires_grad = False
        if self.frozen_stages >= 1:
            for i in range(self.frozen_stages):
                for p in self.layers[i].parameters():
                    p.requires_grad = False

    @staticmethod
    def _init_module(m):
        """video_swin_transformer.py:578-585 / :643-650: Linear weights trunc_normal(std .02), biases 0; LayerNorm 1 / 0."""
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def inflate_weights(self, logger=print):
        """video_swin_transformer.py:566-632: load a 2-D Swin checkpoint ({'model': state_dict}) into this 3-D model —
        relative_position_index / attn_mask entries dropped (re-initialised here), patch_embed.proj.weight repeated
        over the patch depth and divided by it, relative_position_bias_table bicubic-resized to (2Wh-1, 2Ww-1) when
        its side differs and repeated 2Wd-1 times; strict=False.  Loaded with weights_only=True (tensors only)."""
        self.apply(self._init_module)
        checkpoint = torch.load(self.pretrained, map_location="cpu", weights_only=True)
        state_dict = dict(checkpoint["model"])
        for k in [k for k in state_dict if "relative_position_index" in k or "attn_mask" in k]:
            del state_dict[k]
        pd = self.patch_size[0]
        state_dict["patch_embed.proj.weight"] = state_dict["patch_embed.proj.weight"].unsqueeze(2).repeat(1, 1, pd, 1, 1) / pd
        own = self.state_dict()
        wd, wh, ww = self.window_size
        for k in [k for k in state_dict if "relative_position_bias_table" in k]:
            t = state_dict[k]
            L1, nH1 = t.size()
            nH2 = own[k].size(1)
            L2 = (2 * wh - 1) * (2 * ww - 1)
            if nH1 != nH2:
                logger(f"Error in loading {k}, passing")
            elif L1 != L2:
                S1 = int(L1 ** 0.5)
                t = torch.nn.functional.interpolate(t.permute(1, 0).view(1, nH1, S1, S1), size=(2 * wh - 1, 2 * ww - 1),
                                                    mode="bicubic").view(nH2, L2).permute(1, 0)
            state_dict[k] = t.repeat(2 * wd - 1, 1)
        msg = self.load_state_dict(state_dict, strict=False)
        logger(msg)
        logger(f"=> loaded successfully '{self.pretrained}'")

    def init_weights(self, pretrained=None):
        """video_swin_transformer.py:634-666: re-initialise (Linear trunc_normal, LayerNorm 1 / 0), then inflate a 2-D
        checkpoint (pretrained2d) or load a 3-D one ({'state_dict' | plain} state_dict, 'module.' / 'backbone.'
        prefixes stripped, strict=False: mmcv load_checkpoint's behaviour for this backbone)."""
        if pretrained:
            self.pretrained = pretrained
        if isinstance(self.pretrained, str):
            self.apply(self._init_module)
            if self.pretrained2d:
                self.inflate_weights()
            else:
                ck = torch.load(self.pretrained, map_location="cpu", weights_only=True)
                sd = ck.get("state_dict", ck) if isinstance(ck, dict) else ck
                sd = {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}
                if any(k.startswith("backbone.") for k in sd):
                    sd = {k[9:]: v for k, v in sd.items() if k.startswith("backbone.")}
                self.load_state_dict(sd, strict=False)
        elif self.pretrained is None:
            self.apply(self._init_module)
        else:
            raise TypeError("pretrained must be a str or None")

    def forward_tokens(self, x, layout="bcthw"):
        """-> final-LN channels-last [B, D', H', W', 8C] in the compute dtype."""
        x = self.patch_embed.tokens(x, layout)
        for layer in self.layers:
            x = layer.forward_tokens(x)
        return Fn.layer_norm(x, self.norm)

    def forward(self, x):
        return self.forward_tokens(x).permute(0, 4, 1, 2, 3).contiguous()

    def train(self, mode=True):
        """Q2: the reference returns None here; we return self (never chain either way)."""
        super().train(mode)
        self._freeze_stages()
        return self


class PoolingMLP(nn.Module):
    """video_swin_transformer.py:688-731 with PoolingMethod 'mean' (the 'Attention' variant's
    TransformerEncoder head is not built): classify = Mlp(mean over D,H,W), feat = mean over H,W -> [B,D,C].
    Takes the backbone's channels-last tokens [B, D, H, W, C]."""

    def __init__(self, args, in_feature, num_hidden=128, num_classes=2, PoolingMethod='mean'):
        super().__init__()
        if PoolingMethod not in (None, 'mean'):
            raise NotImplementedError("PoolingMLP: only the 'mean' pooling is built")
        self.Pooling = 'mean'
        self.mlp = Mlp(in_feature, num_hidden, num_classes, drop=getattr(args, "classify_drop", 0.0))

    def forward(self, t):
        B, D, H, W, C = t.shape
        classify = self.mlp(Fn.RowMeanFn.apply(t.reshape(-1, C), B))
        feat = t.float().mean(dim=(2, 3))
        return classify.squeeze(), feat


class VideoClassifier(nn.Module):
    """video_swin_transformer.py:734-793 (video modality): SwinTransformer3D -> PoolingMLP -> sigmoid.
    Returns the probability only: the reference returns (prob, feat[B,D,C]), a tuple its own Trainer's
    BCELoss cannot take (src/trainer.py:132).  The reference builds Swin with depths 2,2,18,2 / window 8x7x7 /
    drop_path 0.1 and loads args.video_pretrained_dir unconditionally (Q8, absent here): `backbone`
    overrides the architecture, and no checkpoint is read.  Input [B,T,C,H,W] as the dataset yields
    it (the reference never permutes, Q8)."""

    def __init__(self, args, backbone=None, num_classes=2, num_hiddens=None):
        super().__init__()
        self.videoSwinT = backbone or SwinTransformer3D(embed_dim=96, depths=[2, 2, 18, 2], num_heads=[3, 6, 12, 24],
                                                        patch_size=(2, 4, 4), window_size=(8, 7, 7),
                                                        drop_path_rate=0.1, patch_norm=True)
        self.pool = getattr(args, "video_pool", None)
        self.classsifier = PoolingMLP(args, self.videoSwinT.num_features,
                                      num_hiddens or getattr(args, "num_hiddens", 128), num_classes, self.pool)
        self.prob = nn.Sigmoid()

    def forward(self, x):
        t = self.videoSwinT.forward_tokens(x, layout="btchw")
        classify, feat = self.classsifier(t)
        return self.prob(classify.float())


class VSTFeat(nn.Module):
    """Video slot of the north-star FusionModel: the dataset's
    [B,T,C,H,W] clip read in place (strided im2col, no permute copy) ->
    SwinTransformer3D tokens -> mean over (D,H,W) == PoolingMLP 'mean'
    (video_swin_transformer.py:715) -> [B, 8C] fp32."""

    def __init__(self, vst):
        super().__init__()
        self.vst = vst

    def forward(self, x):
        t = self.vst.forward_tokens(x, layout="btchw")
        B = t.shape[0]
        return Fn.RowMeanFn.apply(t.reshape(-1, t.shape[-1]), B)
