"""Oracle: wav2vec2-base (transformers 5.15.0 Wav2Vec2Model) + Audio2D, fp32 CPU.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  wav2vec2 is third-party
(transformers; the reference pins no version, its checkpoint config says
4.7.0.dev0): the restatement follows the container's transformers 5.15.0
``models/wav2vec2/modeling_wav2vec2.py`` (HF/ below) and is pinned by the golden
fixtures generated from it.  Deterministic configuration only: every dropout,
LayerDrop and SpecAugment off (Q12).  Parameter names equal HF's state_dict.
"""
import json

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.utils import parametrizations


class W2VConfig:
    def __init__(self, path=None, **kw):
        d = {}
        if path:
            with open(path) as f:
                d = json.load(f)
        d.update(kw)
        self.conv_dim = d.get("conv_dim", [512] * 7)
        self.conv_kernel = d.get("conv_kernel", [10, 3, 3, 3, 3, 2, 2])
        self.conv_stride = d.get("conv_stride", [5, 2, 2, 2, 2, 2, 2])
        self.hidden = d.get("hidden_size", 768)
        self.heads = d.get("num_attention_heads", 12)
        self.inter = d.get("intermediate_size", 3072)
        self.layers = d.get("num_hidden_layers", 12)
        self.pos_k = d.get("num_conv_pos_embeddings", 128)
        self.pos_g = d.get("num_conv_pos_embedding_groups", 16)
        self.eps = d.get("layer_norm_eps", 1e-5)
        self.mask_time_prob = d.get("mask_time_prob", 0.05)


class ConvLayer(nn.Module):
    """HF/:253-272 (no-norm conv + GELU) and :302-323 (conv0 + GroupNorm(512,512) + GELU)."""
    def __init__(self, cin, cout, k, s, group_norm):
        super().__init__()
        self.conv = nn.Conv1d(cin, cout, k, s, bias=False)
        self.layer_norm = nn.GroupNorm(cout, cout, affine=True) if group_norm else None

    def forward(self, x):
        x = self.conv(x)
        if self.layer_norm is not None:
            x = self.layer_norm(x)
        return F.gelu(x)


class FeatureEncoder(nn.Module):
    """HF/:382-419."""
    def __init__(self, c):
        super().__init__()
        dims = [1] + list(c.conv_dim)
        self.conv_layers = nn.ModuleList([
            ConvLayer(dims[i], dims[i + 1], c.conv_kernel[i], c.conv_stride[i], i == 0) for i in range(len(c.conv_dim))])

    def forward(self, wave):
        x = wave[:, None]
        for layer in self.conv_layers:
            x = layer(x)
        return x


class FeatureProjection(nn.Module):
    """HF/:422-435: LN(512) -> Linear(512->768)."""
    def __init__(self, c):
        super().__init__()
        self.layer_norm = nn.LayerNorm(c.conv_dim[-1], eps=c.eps)
        self.projection = nn.Linear(c.conv_dim[-1], c.hidden)

    def forward(self, x):
        n = self.layer_norm(x)
        return self.projection(n), n


class PosConv(nn.Module):
    """HF/:326-380: weight-norm(dim=2) grouped Conv1d(k=128, pad 64, groups 16),
    drop the last frame (SamePad), GELU."""
    def __init__(self, c):
        super().__init__()
        conv = nn.Conv1d(c.hidden, c.hidden, c.pos_k, padding=c.pos_k // 2, groups=c.pos_g)
        self.conv = parametrizations.weight_norm(conv, name="weight", dim=2)
        self.remove = 1 if c.pos_k % 2 == 0 else 0

    def forward(self, x):              # x [B, T, C]
        y = self.conv(x.transpose(1, 2))
        if self.remove:
            y = y[:, :, :-self.remove]
        return F.gelu(y).transpose(1, 2)


class Attention(nn.Module):
    """HF/:466-548 with eager_attention_forward :438-463: softmax(q k^T * hd^-0.5) v."""
    def __init__(self, c):
        super().__init__()
        self.h, self.hd = c.heads, c.hidden // c.heads
        self.k_proj = nn.Linear(c.hidden, c.hidden)
        self.v_proj = nn.Linear(c.hidden, c.hidden)
        self.q_proj = nn.Linear(c.hidden, c.hidden)
        self.out_proj = nn.Linear(c.hidden, c.hidden)

    def forward(self, x):
        B, T, C = x.shape
        sh = lambda t: t.view(B, T, self.h, self.hd).transpose(1, 2)  # noqa: E731
        q, k, v = sh(self.q_proj(x)), sh(self.k_proj(x)), sh(self.v_proj(x))
        p = torch.softmax(torch.matmul(q, k.transpose(2, 3)) * self.hd ** -0.5, dim=-1)
        return self.out_proj(torch.matmul(p, v).transpose(1, 2).reshape(B, T, C))


class FeedForward(nn.Module):
    """HF/:551-573."""
    def __init__(self, c):
        super().__init__()
        self.intermediate_dense = nn.Linear(c.hidden, c.inter)
        self.output_dense = nn.Linear(c.inter, c.hidden)

    def forward(self, x):
        return self.output_dense(F.gelu(self.intermediate_dense(x)))


class EncoderLayer(nn.Module):
    """HF/:575-608 (post-LN, do_stable_layer_norm=false)."""
    def __init__(self, c):
        super().__init__()
        self.attention = Attention(c)
        self.layer_norm = nn.LayerNorm(c.hidden, eps=c.eps)
        self.feed_forward = FeedForward(c)
        self.final_layer_norm = nn.LayerNorm(c.hidden, eps=c.eps)

    def forward(self, x):
        x = self.layer_norm(x + self.attention(x))
        return self.final_layer_norm(x + self.feed_forward(x))


class Encoder(nn.Module):
    """HF/:657-727 (no attention mask: synthetic clips share one length, Q13)."""
    def __init__(self, c):
        super().__init__()
        self.pos_conv_embed = PosConv(c)
        self.layer_norm = nn.LayerNorm(c.hidden, eps=c.eps)
        self.layers = nn.ModuleList([EncoderLayer(c) for _ in range(c.layers)])

    def forward(self, x):
        x = self.layer_norm(x + self.pos_conv_embed(x))
        for layer in self.layers:
            x = layer(x)
        return x


class Wav2Vec2Model(nn.Module):
    """HF/:1244-1380 forward: features -> projection -> (SpecAugment: off) -> encoder."""
    def __init__(self, c):
        super().__init__()
        self.config = c
        self.feature_extractor = FeatureEncoder(c)
        self.feature_projection = FeatureProjection(c)
        if c.mask_time_prob > 0:
            self.masked_spec_embed = nn.Parameter(torch.zeros(c.hidden))
        self.encoder = Encoder(c)

    def forward(self, wave):
        f = self.feature_extractor(wave).transpose(1, 2)
        h, ext = self.feature_projection(f)
        return {"last_hidden_state": self.encoder(h), "extract_features": ext}


class Audio2D(nn.Module):
    """src/models/audioTransformer.py:5-30 with use_feat=True: mean over frames
    (AdaptiveAvgPool2d((1,768))) then dropout(p=swin_drop, always on, Q9)."""
    def __init__(self, wav_model, swin_drop=0.0, num_classes=1):
        super().__init__()
        self.wav_model = wav_model
        self.classifier = nn.Linear(512, num_classes)      # Q10: created, never used
        self.swin_drop = swin_drop

    def forward(self, x):
        f = self.wav_model(x)["last_hidden_state"].mean(dim=1)
        return F.dropout(f, self.swin_drop) if self.swin_drop > 0 else f
