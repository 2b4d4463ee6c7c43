"""Oracle: Video Swin Transformer 3D restated in fp32 torch on CPU.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Parameter names and shapes
equal the reference's state_dict keys; the arithmetic is restated from
/root/reference/src/models/video_swin_transformer.py (cited per function) with
the window partition / cyclic shift expressed as explicit gathers so that it is
independent of the reference's view/permute formulation.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def clamp_window(dhw, window, shift):
    """get_window_size (video_swin_transformer.py:75-88): a dimension no larger
    than the window uses the whole dimension as window and is never shifted (Q6)."""
    ws = [min(s, w) for s, w in zip(dhw, window)]
    ss = [0 if d <= w else sh for d, w, sh in zip(dhw, window, shift)]
    return tuple(ws), tuple(ss)


def region_labels(Dp, Hp, Wp, ws, ss):
    """compute_mask region ids (video_swin_transformer.py:319-333) per padded
    position: slices [0,P-w), [P-w,P-s), [P-s,P) -> 0,1,2; a zero shift makes the
    last slice the whole axis, i.e. one region (label 2)."""
    def axis(P, w, s):
        lab = torch.full((P,), 2, dtype=torch.long)
        if s > 0:
            idx = torch.arange(P)
            lab = torch.where(idx < P - w, 0, torch.where(idx < P - s, 1, 2))
        return lab
    ld, lh, lw = axis(Dp, ws[0], ss[0]), axis(Hp, ws[1], ss[1]), axis(Wp, ws[2], ss[2])
    return ld[:, None, None] * 9 + lh[None, :, None] * 3 + lw[None, None, :]


def window_token_index(Dp, Hp, Wp, ws):
    """[nW, N] flat index into the padded (shifted) volume for window_partition
    (video_swin_transformer.py:42-54): windows raster over (d,h,w), tokens raster
    inside the window."""
    nd, nh, nw = Dp // ws[0], Hp // ws[1], Wp // ws[2]
    wd, wh, ww = torch.meshgrid(torch.arange(nd), torch.arange(nh), torch.arange(nw), indexing="ij")
    td, th, tw = torch.meshgrid(torch.arange(ws[0]), torch.arange(ws[1]), torch.arange(ws[2]), indexing="ij")
    d = wd.reshape(-1, 1) * ws[0] + td.reshape(1, -1)
    h = wh.reshape(-1, 1) * ws[1] + th.reshape(1, -1)
    w = ww.reshape(-1, 1) * ws[2] + tw.reshape(1, -1)
    return (d * Hp + h) * Wp + w


def shift_mask(Dp, Hp, Wp, ws, ss):
    """[nW, N, N] additive mask with 0 / -100.0 (Q4), video_swin_transformer.py:331-332."""
    lab = region_labels(Dp, Hp, Wp, ws, ss).reshape(-1)
    tok = window_token_index(Dp, Hp, Wp, ws)
    lw = lab[tok]
    return torch.where(lw[:, :, None] == lw[:, None, :], 0.0, -100.0).float()


def rpb_index(full_window, N):
    """relative_position_index[:N,:N] (video_swin_transformer.py:118-132,155):
    token ids decoded with the FULL window geometry even when the window was
    clamped (Q3)."""
    Wd, Wh, Ww = full_window
    t = torch.arange(N)
    d, h, w = t // (Wh * Ww), (t // Ww) % Wh, t % Ww
    rd = d[:, None] - d[None, :] + Wd - 1
    rh = h[:, None] - h[None, :] + Wh - 1
    rw = w[:, None] - w[None, :] + Ww - 1
    return (rd * (2 * Wh - 1) + rh) * (2 * Ww - 1) + rw


class Mlp(nn.Module):
    """src/utils.py:242-260 — fc1 -> exact GELU -> fc2 (dropouts are 0 here)."""
    def __init__(self, cin, hidden, cout=None):
        super().__init__()
        self.fc1 = nn.Linear(cin, hidden)
        self.fc2 = nn.Linear(hidden, cout or cin)

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x)))


class WindowAttention3D(nn.Module):
    """video_swin_transformer.py:91-173 (forward :142-173)."""
    def __init__(self, dim, window_size, num_heads):
        super().__init__()
        self.dim, self.window_size, self.num_heads = dim, tuple(window_size), num_heads
        L = (2 * window_size[0] - 1) * (2 * window_size[1] - 1) * (2 * window_size[2] - 1)
        self.relative_position_bias_table = nn.Parameter(torch.zeros(L, num_heads))
        N = window_size[0] * window_size[1] * window_size[2]
        self.register_buffer("relative_position_index", rpb_index(window_size, N))
        self.qkv = nn.Linear(dim, 3 * dim)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x, mask=None):
        B_, N, C = x.shape
        nH, hd = self.num_heads, C // self.num_heads
        qkv = self.qkv(x).view(B_, N, 3, nH, hd)
        q = qkv[:, :, 0].transpose(1, 2) * (hd ** -0.5)          # Q5: scale q first
        k = qkv[:, :, 1].transpose(1, 2)
        v = qkv[:, :, 2].transpose(1, 2)
        s = torch.einsum("bhnd,bhmd->bhnm", q, k)
        bias = self.relative_position_bias_table[rpb_index(self.window_size, N).reshape(-1)]
        s = s + bias.view(N, N, nH).permute(2, 0, 1)[None]
        if mask is not None:
            nW = mask.shape[0]
            s = (s.view(B_ // nW, nW, nH, N, N) + mask[None, :, None]).view(B_, nH, N, N)
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("bhnm,bhmd->bnhd", p, v).reshape(B_, N, C)
        return self.proj(o)


class SwinTransformerBlock3D(nn.Module):
    """video_swin_transformer.py:176-278."""
    def __init__(self, dim, num_heads, window_size, shift_size):
        super().__init__()
        self.window_size, self.shift_size = tuple(window_size), tuple(shift_size)
        self.norm1 = nn.LayerNorm(dim)
        self.attn = WindowAttention3D(dim, window_size, num_heads)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = Mlp(dim, int(dim * 4))

    def attn_part(self, x):
        """forward_part1 (:219-253): LN -> pad (after LN) -> roll(-s) ->
        partition -> W-MSA -> reverse -> roll(+s) -> crop, all as one gather /
        scatter of token rows."""
        B, D, H, W, C = x.shape
        ws, ss = clamp_window((D, H, W), self.window_size, self.shift_size)
        x = F.layer_norm(x, (C,), self.norm1.weight, self.norm1.bias)
        Dp, Hp, Wp = [-(-n // w) * w for n, w in zip((D, H, W), ws)]
        x = F.pad(x, (0, 0, 0, Wp - W, 0, Hp - H, 0, Dp - D))
        tok = window_token_index(Dp, Hp, Wp, ws)                     # shifted-frame positions
        d, h, w = tok // (Hp * Wp), (tok // Wp) % Hp, tok % Wp
        src = (((d + ss[0]) % Dp) * Hp + (h + ss[1]) % Hp) * Wp + (w + ss[2]) % Wp  # roll(-s)
        flat = x.reshape(B, Dp * Hp * Wp, C)
        win = flat[:, src.reshape(-1)].reshape(B * tok.shape[0], tok.shape[1], C)
        mask = shift_mask(Dp, Hp, Wp, ws, ss) if any(s > 0 for s in ss) else None
        y = self.attn(win, mask).reshape(B, -1, C)
        out = torch.zeros_like(flat).index_copy(1, src.reshape(-1), y)
        return out.view(B, Dp, Hp, Wp, C)[:, :D, :H, :W]

    def forward(self, x):
        x = x + self.attn_part(x)
        return x + self.mlp(F.layer_norm(x, (x.shape[-1],), self.norm2.weight, self.norm2.bias))


class PatchMerging(nn.Module):
    """video_swin_transformer.py:281-316 (Q7 gather order x0,x1,x2,x3)."""
    def __init__(self, dim):
        super().__init__()
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = nn.LayerNorm(4 * dim)

    def forward(self, x):
        B, D, H, W, C = x.shape
        x = F.pad(x, (0, 0, 0, W % 2, 0, H % 2))
        parts = [x[:, :, i::2, j::2] for (i, j) in ((0, 0), (1, 0), (0, 1), (1, 1))]
        return self.reduction(self.norm(torch.cat(parts, -1)))


class PatchEmbed3D(nn.Module):
    """video_swin_transformer.py:420-460: zero-pad to the patch grid, Conv3d with
    kernel = stride = patch, LayerNorm over channels."""
    def __init__(self, patch_size=(2, 4, 4), in_chans=3, embed_dim=96, norm=True):
        super().__init__()
        self.patch_size = tuple(patch_size)
        self.proj = nn.Conv3d(in_chans, embed_dim, self.patch_size, self.patch_size)
        self.norm = nn.LayerNorm(embed_dim) if norm else None

    def forward(self, x):
        _, _, D, H, W = x.shape
        pd, ph, pw = self.patch_size
        x = F.pad(x, (0, (-W) % pw, 0, (-H) % ph, 0, (-D) % pd))
        x = self.proj(x)
        if self.norm is not None:
            x = self.norm(x.permute(0, 2, 3, 4, 1)).permute(0, 4, 1, 2, 3)
        return x


class BasicLayer(nn.Module):
    """video_swin_transformer.py:336-417 (blocks alternate shift 0 / window//2)."""
    def __init__(self, dim, depth, num_heads, window_size, downsample):
        super().__init__()
        self.window_size = tuple(window_size)
        shift = tuple(w // 2 for w in window_size)
        self.blocks = nn.ModuleList([
            SwinTransformerBlock3D(dim, num_heads, window_size, (0, 0, 0) if i % 2 == 0 else shift)
            for i in range(depth)])
        self.downsample = PatchMerging(dim) if downsample else None

    def forward(self, x):            # x: [B, C, D, H, W]
        x = x.permute(0, 2, 3, 4, 1)
        for blk in self.blocks:
            x = blk(x)
        if self.downsample is not None:
            x = self.downsample(x)
        return x.permute(0, 4, 1, 2, 3)


class SwinTransformer3D(nn.Module):
    """video_swin_transformer.py:462-686 (forward :668-681); dropouts and
    DropPath are identity (rates 0 for parity)."""
    def __init__(self, patch_size=(2, 4, 4), in_chans=3, embed_dim=96, depths=(2, 2, 6, 2),
                 num_heads=(3, 6, 12, 24), window_size=(8, 7, 7), patch_norm=True, **_):
        super().__init__()
        self.patch_embed = PatchEmbed3D(patch_size, in_chans, embed_dim, patch_norm)
        self.layers = nn.ModuleList([
            BasicLayer(embed_dim * 2 ** i, depths[i], num_heads[i], window_size, i < len(depths) - 1)
            for i in range(len(depths))])
        self.num_features = embed_dim * 2 ** (len(depths) - 1)
        self.norm = nn.LayerNorm(self.num_features)

    def forward(self, x):
        x = self.patch_embed(x)
        for layer in self.layers:
            x = layer(x)
        x = self.norm(x.permute(0, 2, 3, 4, 1))
        return x.permute(0, 4, 1, 2, 3)


class VSTFeat(nn.Module):
    """Video slot of the north-star FusionModel: permute the
    dataset's [B,T,C,H,W] to [B,C,T,H,W], run the VST, mean over (D,H,W) as
    PoolingMLP 'mean' does (video_swin_transformer.py:715)."""
    def __init__(self, vst):
        super().__init__()
        self.vst = vst

    def forward(self, x):
        return self.vst(x.permute(0, 2, 1, 3, 4)).mean(dim=[2, 3, 4])
