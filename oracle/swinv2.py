"""Oracle: SwinTransformerV2 (mel branch, use_feat=True) restated in fp32 CPU torch.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates
/root/reference/src/models/swin_transformer2d.py (cited per class).  Names equal
the reference state_dict keys.  DropPath / dropouts are identity (rates 0).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .vst import Mlp


def coords_table(ws, pretrained_ws):
    """swin_transformer2d.py:94-108: log-spaced relative coordinates, [1,2W-1,2W-1,2]."""
    r = torch.arange(-(ws - 1), ws, dtype=torch.float32)
    t = torch.stack(torch.meshgrid([r, r], indexing="ij")).permute(1, 2, 0).contiguous()[None]
    den = (pretrained_ws - 1) if pretrained_ws > 0 else (ws - 1)
    t = t / den * 8
    return torch.sign(t) * torch.log2(t.abs() + 1.0) / math.log2(8)


def rel_index_2d(ws):
    """swin_transformer2d.py:112-121."""
    t = torch.arange(ws * ws)
    h, w = t // ws, t % ws
    return (h[:, None] - h[None, :] + ws - 1) * (2 * ws - 1) + (w[:, None] - w[None, :] + ws - 1)


def window_tokens_2d(H, W, ws):
    nh, nw = H // ws, W // ws
    wh, ww = torch.meshgrid(torch.arange(nh), torch.arange(nw), indexing="ij")
    th, tw = torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")
    h = wh.reshape(-1, 1) * ws + th.reshape(1, -1)
    w = ww.reshape(-1, 1) * ws + tw.reshape(1, -1)
    return h, w


def shift_mask_2d(H, W, ws, s):
    """swin_transformer2d.py:246-264 (0 / -100)."""
    def lab(P):
        i = torch.arange(P)
        return torch.where(i < P - ws, 0, torch.where(i < P - s, 1, 2))
    L = lab(H)[:, None] * 3 + lab(W)[None, :]
    h, w = window_tokens_2d(H, W, ws)
    lw = L[h, w]
    return torch.where(lw[:, :, None] == lw[:, None, :], 0.0, -100.0)


class WindowAttention(nn.Module):
    """swin_transformer2d.py:67-184: cosine attention, clamped logit scale,
    continuous position bias 16*sigmoid(cpb_mlp(coords))."""
    def __init__(self, dim, ws, num_heads, pretrained_ws):
        super().__init__()
        self.ws, self.nH = ws, num_heads
        self.logit_scale = nn.Parameter(torch.log(10 * torch.ones(num_heads, 1, 1)))
        self.cpb_mlp = nn.Sequential(nn.Linear(2, 512, bias=True), nn.ReLU(inplace=True),
                                     nn.Linear(512, num_heads, bias=False))
        self.register_buffer("relative_coords_table", coords_table(ws, pretrained_ws))
        self.register_buffer("relative_position_index", rel_index_2d(ws))
        self.qkv = nn.Linear(dim, 3 * dim, bias=False)
        self.q_bias = nn.Parameter(torch.zeros(dim))
        self.v_bias = nn.Parameter(torch.zeros(dim))
        self.proj = nn.Linear(dim, dim)

    def bias_table(self):
        """[nH, N, N] = 16*sigmoid(cpb_mlp(table)[index])."""
        N = self.ws * self.ws
        t = self.cpb_mlp(self.relative_coords_table).view(-1, self.nH)
        return 16 * torch.sigmoid(t[rel_index_2d(self.ws).reshape(-1)].view(N, N, self.nH).permute(2, 0, 1))

    def forward(self, x, mask=None):
        B_, N, C = x.shape
        b = torch.cat((self.q_bias, torch.zeros_like(self.v_bias), self.v_bias))
        qkv = F.linear(x, self.qkv.weight, b).view(B_, N, 3, self.nH, -1).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        s = F.normalize(q, dim=-1) @ F.normalize(k, dim=-1).transpose(-2, -1)
        s = s * torch.clamp(self.logit_scale, max=math.log(1.0 / 0.01)).exp()
        s = s + self.bias_table()[None]
        if mask is not None:
            nW = mask.shape[0]
            s = (s.view(B_ // nW, nW, self.nH, N, N) + mask[None, :, None]).view(B_, self.nH, N, N)
        return self.proj((torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B_, N, C))


class SwinTransformerBlock(nn.Module):
    """swin_transformer2d.py:187-291: post-norm residuals x + LN(attn(x)), x + LN(mlp(x))."""
    def __init__(self, dim, res, num_heads, ws, shift, pretrained_ws):
        super().__init__()
        self.res = res
        if min(res) <= ws:
            shift, ws = 0, min(res)
        self.ws, self.shift = ws, shift
        self.norm1 = nn.LayerNorm(dim)
        self.attn = WindowAttention(dim, ws, num_heads, pretrained_ws)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = Mlp(dim, dim * 4)
        self.register_buffer("attn_mask", shift_mask_2d(res[0], res[1], ws, shift) if shift > 0 else None)

    def forward(self, x):
        H, W = self.res
        B, L, C = x.shape
        h, w = window_tokens_2d(H, W, self.ws)
        src = ((h + self.shift) % H) * W + (w + self.shift) % W
        win = x[:, src.reshape(-1)].reshape(-1, self.ws * self.ws, C)
        y = self.attn(win, self.attn_mask).reshape(B, -1, C)
        y = torch.zeros_like(x).index_copy(1, src.reshape(-1), y)
        x = x + self.norm1(y)
        return x + self.norm2(self.mlp(x))


class PatchMerging(nn.Module):
    """swin_transformer2d.py:327-364: gather x0..x3, Linear(4C->2C), LN(2C)."""
    def __init__(self, res, dim):
        super().__init__()
        self.res = res
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = nn.LayerNorm(2 * dim)

    def forward(self, x):
        H, W = self.res
        B, L, C = x.shape
        x = x.view(B, H, W, C)
        parts = [x[:, i::2, j::2] for (i, j) in ((0, 0), (1, 0), (0, 1), (1, 1))]
        return self.norm(self.reduction(torch.cat(parts, -1).view(B, -1, 4 * C)))


class BasicLayer(nn.Module):
    def __init__(self, dim, res, depth, num_heads, ws, downsample, pretrained_ws):
        super().__init__()
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim, res, num_heads, ws, 0 if i % 2 == 0 else ws // 2, pretrained_ws)
            for i in range(depth)])
        self.downsample = PatchMerging(res, dim) if downsample else None

    def forward(self, x):
        for b in self.blocks:
            x = b(x)
        return self.downsample(x) if self.downsample is not None else x


class PatchEmbed(nn.Module):
    """swin_transformer2d.py:440-483 (Conv2d k=s=4, LN)."""
    def __init__(self, patch, cin, dim):
        super().__init__()
        self.proj = nn.Conv2d(cin, dim, patch, patch)
        self.norm = nn.LayerNorm(dim)

    def forward(self, x):
        return self.norm(self.proj(x).flatten(2).transpose(1, 2))


class SwinTransformerV2(nn.Module):
    """swin_transformer2d.py:486-629 with use_feat=True: forward_features ->
    final LN -> mean over tokens (AdaptiveAvgPool1d)."""
    def __init__(self, img_size=224, patch_size=4, in_chans=3, embed_dim=96, depths=(2, 2, 6, 2),
                 num_heads=(3, 6, 12, 24), window_size=7, pretrained_window_sizes=(0, 0, 0, 0), **_):
        super().__init__()
        self.patch_embed = PatchEmbed(patch_size, in_chans, embed_dim)
        r = img_size // patch_size
        self.layers = nn.ModuleList([
            BasicLayer(embed_dim * 2 ** i, (r // 2 ** i, r // 2 ** i), depths[i], num_heads[i], window_size,
                       i < len(depths) - 1, pretrained_window_sizes[i])
            for i in range(len(depths))])
        self.norm = nn.LayerNorm(embed_dim * 2 ** (len(depths) - 1))

    def forward(self, x):
        x = self.patch_embed(x)
        for layer in self.layers:
            x = layer(x)
        return self.norm(x).mean(dim=1)
