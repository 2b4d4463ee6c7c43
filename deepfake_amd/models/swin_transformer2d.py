"""SwinTransformerV2 (mel-spectrogram branch) on MI355X — drop-in for
/root/reference/src/models/swin_transformer2d.py (classes, constructor
signatures, state_dict keys incl. the persistent ``attn_mask`` buffers).

A 2-D window is the 3-D window kernel with depth 1: token-major rows
[B, H, W, C], shift/partition/reverse as index arithmetic, the 0/-100 shift
mask from region labels in-kernel.  Cosine attention = dfk_cosine_qk (q,k
normalised, q scaled by exp(clamp(logit_scale))) + window attention with the
16*sigmoid(cpb_mlp) table as the relative-position bias.  Post-norm residuals
x + LN(attn(x)), x + LN(mlp(x)) (:288-291).
"""
import math
import os

import numpy as np
import torch
import torch.nn as nn

from .. import functional as Fn
from .. import rng


def to_2tuple(x):
    return tuple(x) if isinstance(x, (list, tuple)) else (x, x)


class Mlp(nn.Module):
    """swin_transformer2d.py:16-32."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)   # module tree parity; the masks are the two device sites below
        self.sites = (rng.Drop(drop), rng.Drop(drop)) if drop > 0 else None   # after the GELU, after fc2

    def drop_specs(self):
        if self.sites is None or not self.training:
            return None, None
        return self.sites[0].spec(), self.sites[1].spec()


def window_partition(x, window_size):
    """swin_transformer2d.py:35-47 (API utility)."""
    B, H, W, C = x.shape
    x = x.view(B, H // window_size, window_size, W // window_size, window_size, C)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(-1, window_size, window_size, C)


def window_reverse(windows, window_size, H, W):
    """swin_transformer2d.py:50-64."""
    B = int(windows.shape[0] / (H * W / window_size / window_size))
    x = windows.view(B, H // window_size, W // window_size, window_size, window_size, -1)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(B, H, W, -1)


class WindowAttention(nn.Module):
    """swin_transformer2d.py:67-184 (cosine attention + continuous position bias)."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=True, attn_drop=0., proj_drop=0.,
                 pretrained_window_size=[0, 0]):
        super().__init__()
        # attn_drop (:176, softmax probabilities, in the attention kernel) and proj_drop (:182, proj epilogue)
        # as device dropout sites, created only when p > 0
        self.attn_drop = rng.Drop(attn_drop) if attn_drop > 0 else None
        self.proj_drop = rng.Drop(proj_drop) if proj_drop > 0 else None
        self.dim, self.window_size, self.pretrained_window_size = dim, window_size, pretrained_window_size
        self.num_heads = num_heads
        self.logit_scale = nn.Parameter(torch.log(10 * torch.ones((num_heads, 1, 1))), requires_grad=True)
        self.cpb_mlp = nn.Sequential(nn.Linear(2, 512, bias=True), nn.ReLU(inplace=True),
                                     nn.Linear(512, num_heads, bias=False))
        rh = torch.arange(-(window_size[0] - 1), window_size[0], dtype=torch.float32)
        rw = torch.arange(-(window_size[1] - 1), window_size[1], dtype=torch.float32)
        table = torch.stack(torch.meshgrid([rh, rw], indexing="ij")).permute(1, 2, 0).contiguous().unsqueeze(0)
        den = pretrained_window_size if pretrained_window_size[0] > 0 else window_size
        table[:, :, :, 0] /= (den[0] - 1)
        table[:, :, :, 1] /= (den[1] - 1)
        table *= 8
        table = torch.sign(table) * torch.log2(torch.abs(table) + 1.0) / np.log2(8)
        self.register_buffer("relative_coords_table", table)
        ch, cw = torch.arange(window_size[0]), torch.arange(window_size[1])
        coords = torch.flatten(torch.stack(torch.meshgrid([ch, cw], indexing="ij")), 1)
        rel = (coords[:, :, None] - coords[:, None, :]).permute(1, 2, 0).contiguous()
        rel[:, :, 0] += window_size[0] - 1
        rel[:, :, 1] += window_size[1] - 1
        rel[:, :, 0] *= 2 * window_size[1] - 1
        self.register_buffer("relative_position_index", rel.sum(-1))
        self.qkv = nn.Linear(dim, dim * 3, bias=False)
        if qkv_bias:
            self.q_bias = nn.Parameter(torch.zeros(dim))
            self.v_bias = nn.Parameter(torch.zeros(dim))
        else:
            self.q_bias = self.v_bias = None
        self.proj = nn.Linear(dim, dim)

    def bias_table(self):
        """[(2Wh-1)(2Ww-1), nH] fp32 = 16*sigmoid(cpb_mlp(coords)) (:159-164), indexed in-kernel."""
        fc1, fc2 = self.cpb_mlp[0], self.cpb_mlp[2]
        return Fn.CPBBiasFn.apply(self.relative_coords_table, fc1.weight, fc1.bias, fc2.weight)

    def flat_groups(self):
        """ParamStore adjacency: q_bias, a C-element zero gap, v_bias -> the [3C] qkv bias in place."""
        return [[self.q_bias, self.dim, self.v_bias]] if self.q_bias is not None else []

    def core(self, x2d, dims, ws, shift, skip=False):
        """x2d [rows, C] -> attention output [rows, C] before proj (skip=True: and an alias of x2d for the
        block's residual, whose gradient joins the qkv dX GEMM)."""
        C = self.dim
        hd = C // self.num_heads
        xs = x2d
        if self.q_bias is not None:   # qkv bias = cat(q_bias, 0, v_bias) (:151-153): a gapped adjacency group
            qkv = Fn.linear_group(x2d, (self.qkv.weight,), (self.q_bias, C, self.v_bias), skip=skip)
            if skip:
                qkv, xs = qkv
        else:
            qkv = Fn.linear(x2d, self.qkv.weight)
        ad = self.attn_drop.spec() if self.attn_drop is not None and self.training else None
        # logit_scale's gradient: sum dS * score taken in fp32 inside the attention backward (dfk_wattn_bwd_args
        # .dscore), handed to the cosine backward through a per-module buffer
        dsc = Fn.dscore_buffer(self, qkv, self.num_heads, ad) if self.logit_scale.requires_grad else None
        qkv = Fn.CosineQKFn.apply(qkv, self.logit_scale, self.num_heads, hd, math.log(1. / 0.01), dsc)
        geo = (dims, (1, ws, ws), (1, self.window_size[0], self.window_size[1]), (0, shift, shift),
               self.num_heads, hd, 1.0)
        tab = self._cpb if getattr(self, "_cpb", None) is not None else self.bias_table()
        out = Fn.window_attention(qkv, tab, None, geo, drop=ad, dscore=dsc)
        return (out, xs) if skip else out


class SwinTransformerBlock(nn.Module):
    """swin_transformer2d.py:187-291."""

    def __init__(self, dim, input_resolution, num_heads, window_size=7, shift_size=0, mlp_ratio=4., qkv_bias=True,
                 drop=0., attn_drop=0., drop_path=0., act_layer=nn.GELU, norm_layer=nn.LayerNorm,
                 pretrained_window_size=0):
        super().__init__()
        self.dim, self.input_resolution, self.num_heads = dim, input_resolution, num_heads
        self.window_size, self.shift_size, self.mlp_ratio = window_size, shift_size, mlp_ratio
        if min(self.input_resolution) <= self.window_size:
            self.shift_size = 0
            self.window_size = min(self.input_resolution)
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, window_size=to_2tuple(self.window_size), num_heads=num_heads,
                                    qkv_bias=qkv_bias, attn_drop=attn_drop, proj_drop=drop,
                                    pretrained_window_size=to_2tuple(pretrained_window_size))
        self.drop_path = nn.Identity()
        # timm DropPath is called once per branch: two independent per-sample draws
        self.dp = (rng.Drop(drop_path, mode=2), rng.Drop(drop_path, mode=2)) if drop_path > 0 else None
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)
        if self.shift_size > 0:
            H, W = self.input_resolution
            ws, s = self.window_size, self.shift_size

            def lab(P):
                i = torch.arange(P)
                return torch.where(i < P - ws, 0, torch.where(i < P - s, 1, 2))
            img = (lab(H)[:, None] * 3 + lab(W)[None, :]).float()[None, :, :, None]
            mw = window_partition(img, ws).view(-1, ws * ws)
            d = mw.unsqueeze(1) - mw.unsqueeze(2)
            attn_mask = torch.where(d != 0, -100.0, 0.0)
        else:
            attn_mask = None
        self.register_buffer("attn_mask", attn_mask)

    def forward(self, x):
        H, W = self.input_resolution
        B, L, C = x.shape
        assert L == H * W, "input feature has wrong size"
        x2 = x.reshape(-1, C)
        a, x2s = self.attn.core(x2, (B, 1, H, W), self.window_size, self.shift_size, skip=True)
        pd = self.attn.proj_drop.spec() if self.attn.proj_drop is not None and self.training else None
        a = Fn.linear(a, self.attn.proj.weight, self.attn.proj.bias, drop=pd)
        on = self.dp is not None and self.training
        dp = (self.dp[0].spec(L), self.dp[1].spec(L)) if on else (None, None)
        x2 = Fn.layer_norm(a, self.norm1, residual=x2s, drop=dp[0])   # x + DropPath(LN(attn)) (:301)
        da, do = self.mlp.drop_specs()
        m, x2s = Fn.mlp(x2, self.mlp.fc1, self.mlp.fc2, skip=True, drop_act=da, drop_out=do)   # x2's residual
        # gradient joins fc1's dX
        x2 = Fn.layer_norm(m, self.norm2, residual=x2s, drop=dp[1])   # x + DropPath(LN(mlp)) (:304)
        return x2.view(B, L, C)


class PatchMerging(nn.Module):
    """swin_transformer2d.py:327-364: gather x0..x3, Linear(4C->2C), LN(2C)."""

    def __init__(self, input_resolution, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.input_resolution, self.dim = input_resolution, dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = norm_layer(2 * dim)

    def forward(self, x):
        H, W = self.input_resolution
        B, L, C = x.shape
        assert L == H * W and H % 2 == 0 and W % 2 == 0
        m = Fn.PatchMergeFn.apply(x.reshape(-1, C).contiguous(), (B, 1, H, W))
        y = Fn.layer_norm(Fn.linear(m, self.reduction.weight), self.norm)
        return y.view(B, -1, 2 * C)


class BasicLayer(nn.Module):
    """swin_transformer2d.py:367-437."""

    def __init__(self, dim, input_resolution, depth, num_heads, window_size, mlp_ratio=4., qkv_bias=True, drop=0.,
                 attn_drop=0., drop_path=0., norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False,
                 pretrained_window_size=0):
        super().__init__()
        self.dim, self.input_resolution, self.depth = dim, input_resolution, depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim=dim, input_resolution=input_resolution, num_heads=num_heads,
                                 window_size=window_size, shift_size=0 if (i % 2 == 0) else window_size // 2,
                                 mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, drop=drop, attn_drop=attn_drop,
                                 drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                 norm_layer=norm_layer, pretrained_window_size=pretrained_window_size)
            for i in range(depth)])
        self.downsample = downsample(input_resolution, dim=dim, norm_layer=norm_layer) if downsample else None

    def forward(self, x):
        for blk in self.blocks:
            if self.use_checkpoint and self.training and torch.is_grad_enabled():   # :428-429
                x = Fn.checkpoint(blk, x)
            else:
                x = blk(x)
        return self.downsample(x) if self.downsample is not None else x

    def _init_respostnorm(self):
        for blk in self.blocks:
            for n in (blk.norm1, blk.norm2):
                nn.init.constant_(n.bias, 0)
                nn.init.constant_(n.weight, 0)


class PatchEmbed(nn.Module):
    """swin_transformer2d.py:440-483 (Conv2d k=s=patch as im2col + GEMM, LN)."""

    def __init__(self, img_size=224, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        img_size, patch_size = to_2tuple(img_size), to_2tuple(patch_size)
        self.img_size, self.patch_size = img_size, patch_size
        self.patches_resolution = [img_size[0] // patch_size[0], img_size[1] // patch_size[1]]
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.in_chans, self.embed_dim = in_chans, embed_dim
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None
        self.compute_dtype = torch.float32

    def forward(self, x):
        B, C, H, W = x.shape
        assert (H, W) == tuple(self.img_size), "Input image size doesn't match model"
        y = Fn.PatchEmbedFn.apply(x, self.proj.weight, self.proj.bias, "bchw", self.patch_size, self.compute_dtype)
        if self.norm is not None:
            y = Fn.layer_norm(y, self.norm)
        return y.view(B, self.num_patches, self.embed_dim)


class SwinTransformerV2(nn.Module):
    """swin_transformer2d.py:486-629; use_feat=True -> [B, num_features] fp32 features."""

    def __init__(self, img_size=224, patch_size=4, in_chans=3, num_classes=1000, embed_dim=96, depths=[2, 2, 6, 2],
                 num_heads=[3, 6, 12, 24], window_size=7, mlp_ratio=4., qkv_bias=True, drop_rate=0.,
                 attn_drop_rate=0., drop_path_rate=0.1, norm_layer=nn.LayerNorm, ape=False, patch_norm=True,
                 use_checkpoint=False, pretrained_window_sizes=[0, 0, 0, 0], use_feat=False, **kwargs):
        super().__init__()
        if ape:
            raise NotImplementedError("absolute position embedding")
        self.num_classes, self.num_layers, self.embed_dim = num_classes, len(depths), embed_dim
        self.ape, self.patch_norm, self.mlp_ratio, self.use_feat = ape, patch_norm, mlp_ratio, use_feat
        self.num_features = int(embed_dim * 2 ** (self.num_layers - 1))
        self.patch_embed = PatchEmbed(img_size=img_size, patch_size=patch_size, in_chans=in_chans,
                                      embed_dim=embed_dim, norm_layer=norm_layer if patch_norm else None)
        pr = self.patch_embed.patches_resolution
        self.patches_resolution = pr
        self.pos_drop = nn.Identity()
        dpr = [float(x) for x in torch.linspace(0, drop_path_rate, sum(depths))]
        self.layers = nn.ModuleList()
        for i in range(self.num_layers):
            self.layers.append(BasicLayer(
                dim=int(embed_dim * 2 ** i), input_resolution=(pr[0] // (2 ** i), pr[1] // (2 ** i)),
                depth=depths[i], num_heads=num_heads[i], window_size=window_size, mlp_ratio=mlp_ratio,
                qkv_bias=qkv_bias, drop=drop_rate, attn_drop=attn_drop_rate,
                drop_path=dpr[sum(depths[:i]):sum(depths[:i + 1])], norm_layer=norm_layer,
                downsample=PatchMerging if (i < self.num_layers - 1) else None, use_checkpoint=use_checkpoint,
                pretrained_window_size=pretrained_window_sizes[i]))
        self.norm = norm_layer(self.num_features)
        if not use_feat:
            from ..utils import Mlp as HeadMlp
            self.head = HeadMlp(self.num_features, 256, self.num_classes)
        for bly in self.layers:
            bly._init_respostnorm()

    def forward_features(self, x):
        x = self.patch_embed(x)
        # every block's CPB table in one launch each way (parameters only; Fn.cpb_tables), handed to the blocks
        # for this forward only
        attns = [blk.attn for layer in self.layers for blk in layer.blocks]
        if x.is_cuda and os.environ.get("DFK_CPB_MANY", "1") != "0":
            for a, t in zip(attns, Fn.cpb_tables(attns)):
                a._cpb = t
        try:
            for layer in self.layers:
                x = layer(x)
        finally:
            for a in attns:
                a._cpb = None
        B, L, C = x.shape
        x = Fn.layer_norm(x, self.norm)
        return Fn.RowMeanFn.apply(x.reshape(B * L, C), B)

    def forward(self, x):
        x = self.forward_features(x)
        if not self.use_feat:
            return torch.squeeze(torch.sigmoid(self.head(x.to(torch.float32))))
        return x
