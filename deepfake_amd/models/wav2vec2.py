"""wav2vec2-base on MI355X with HF-compatible state_dict keys (drop-in for the
``transformers.Wav2Vec2Model`` the reference builds at train.py:46 and wraps in
Audio2D, audioTransformer.py:5-30).  Restates transformers 5.15.0
models/wav2vec2/modeling_wav2vec2.py (HF/ below) on HIP kernels:

  conv0 + GroupNorm + GELU        dfk_w2v_conv0_*   (HF/:302-323)
  conv1..6 + GELU                 implicit-GEMM conv (HF/:253-272), channels-last
  feature projection LN + Linear  (HF/:422-435)
  weight-normed grouped pos-conv  implicit GEMM per (clip, group), + residual (HF/:326-380,689)
  12 post-LN encoder layers       fused qkv GEMM, whole-sequence attention kernel,
                                  out_proj+residual, LN, FFN(+residual), LN (HF/:575-608)

Training-mode regularisers of the checkpoint config (HF/ sites, all drawn on the
device, deepfake_amd.rng): feat_proj_dropout after the projection GEMM (:433),
SpecAugment time masking with masked_spec_embed (:1272-1317), hidden dropout
after the encoder-input LN (:692), attention-probability dropout inside the
attention kernel (:458), hidden dropout after out_proj and after the FFN output
GEMM (:596,:571), activation dropout after the FFN GELU (:568), all fused into
the producing kernel's epilogue; LayerDrop (:700-706) as per-layer device coins:
a dropped layer still runs (a captured graph cannot branch) but its output is
discarded (torch.where), its gradients are zero and the fused SGD skips its
parameters (as torch's SGD skips grad=None).  config.deterministic() turns all
of them off (the parity setting, Q12).
"""
import json
import os

import torch
import torch.nn as nn
from torch.nn.utils import parametrizations

from .. import functional as Fn
from .. import kernels as K
from .. import rng


class Wav2Vec2Config:
    """The fields of HF Wav2Vec2Config this path reads (config.json of the
    reference checkpoint: checkpoints/wav2vec2-base-960h/config.json)."""

    def __init__(self, **kw):
        self.conv_dim = kw.get("conv_dim", [512] * 7)
        self.conv_kernel = kw.get("conv_kernel", [10, 3, 3, 3, 3, 2, 2])
        self.conv_stride = kw.get("conv_stride", [5, 2, 2, 2, 2, 2, 2])
        self.conv_bias = kw.get("conv_bias", False)
        self.feat_extract_norm = kw.get("feat_extract_norm", "group")
        self.hidden_size = kw.get("hidden_size", 768)
        self.num_attention_heads = kw.get("num_attention_heads", 12)
        self.intermediate_size = kw.get("intermediate_size", 3072)
        self.num_hidden_layers = kw.get("num_hidden_layers", 12)
        self.num_conv_pos_embeddings = kw.get("num_conv_pos_embeddings", 128)
        self.num_conv_pos_embedding_groups = kw.get("num_conv_pos_embedding_groups", 16)
        self.layer_norm_eps = kw.get("layer_norm_eps", 1e-5)
        self.do_stable_layer_norm = kw.get("do_stable_layer_norm", False)
        self.mask_time_prob = kw.get("mask_time_prob", 0.05)
        self.mask_time_length = kw.get("mask_time_length", 10)
        self.mask_time_min_masks = kw.get("mask_time_min_masks", 2)
        self.mask_feature_prob = kw.get("mask_feature_prob", 0.0)
        self.apply_spec_augment = kw.get("apply_spec_augment", True)
        self.layerdrop = kw.get("layerdrop", 0.1)
        for k in ("hidden_dropout", "attention_dropout", "activation_dropout", "feat_proj_dropout"):
            setattr(self, k, kw.get(k, 0.1))

    @classmethod
    def from_json_file(cls, path, **overrides):
        with open(path) as f:
            d = json.load(f)
        d.update(overrides)
        return cls(**d)

    def deterministic(self):
        """Parity / benchmark setting (Q12): dropouts, LayerDrop and SpecAugment off."""
        for k in ("hidden_dropout", "attention_dropout", "activation_dropout", "feat_proj_dropout", "layerdrop",
                  "mask_time_prob", "mask_feature_prob"):
            setattr(self, k, 0.0)
        return self


class _ConvLayer(nn.Module):
    def __init__(self, cin, cout, k, s, group_norm):
        super().__init__()
        self.conv = nn.Conv1d(cin, cout, kernel_size=k, stride=s, bias=False)
        if group_norm:
            self.layer_norm = nn.GroupNorm(num_groups=cout, num_channels=cout, affine=True)
        self.stride = s


class Wav2Vec2FeatureEncoder(nn.Module):
    """HF/:382-419 (feat_extract_norm == "group")."""

    def __init__(self, config):
        super().__init__()
        if config.feat_extract_norm != "group" or config.conv_bias or config.conv_dim[0] != 512 \
                or config.conv_kernel[0] != 10 or config.conv_stride[0] != 5:
            raise NotImplementedError("only the wav2vec2-base feature encoder (group norm, 512x10/5 conv0)")
        dims = [1] + list(config.conv_dim)
        self.conv_layers = nn.ModuleList([
            _ConvLayer(dims[i], dims[i + 1], config.conv_kernel[i], config.conv_stride[i], i == 0)
            for i in range(len(config.conv_dim))])
        self.compute_dtype = torch.float32

    def forward(self, input_values):
        """[B, S] fp32 -> channels-last [B, T, 512] (compute dtype)."""
        l0 = self.conv_layers[0]
        x = Fn.W2VConv0Fn.apply(input_values, l0.conv.weight, l0.layer_norm.weight, l0.layer_norm.bias,
                                l0.layer_norm.eps, self.compute_dtype)
        for layer in self.conv_layers[1:]:
            x = Fn.ConvGeluFn.apply(x, layer.conv.weight, layer.stride)
        return x


class Wav2Vec2FeatureProjection(nn.Module):
    """HF/:422-435."""

    def __init__(self, config):
        super().__init__()
        self.layer_norm = nn.LayerNorm(config.conv_dim[-1], eps=config.layer_norm_eps)
        self.projection = nn.Linear(config.conv_dim[-1], config.hidden_size)
        self.dropout = rng.Drop(config.feat_proj_dropout)

    def forward(self, x):
        n = Fn.layer_norm(x, self.layer_norm)
        d = self.dropout.spec() if self.dropout.active(self.training) else None
        return Fn.linear(n, self.projection.weight, self.projection.bias, drop=d), n


class Wav2Vec2PositionalConvEmbedding(nn.Module):
    """HF/:326-368 (weight-norm dim=2; SamePad drops the last frame)."""

    def __init__(self, config):
        super().__init__()
        conv = nn.Conv1d(config.hidden_size, config.hidden_size, kernel_size=config.num_conv_pos_embeddings,
                         padding=config.num_conv_pos_embeddings // 2, groups=config.num_conv_pos_embedding_groups)
        self.conv = parametrizations.weight_norm(conv, name="weight", dim=2)
        self.groups = config.num_conv_pos_embedding_groups
        if config.num_conv_pos_embeddings % 2:
            raise NotImplementedError("odd num_conv_pos_embeddings")

    def weight(self):
        """weight_norm(dim=2): g * v / ||v|| with the norm over dims (0, 1) — same parameters and state_dict
        keys as the parametrization, composed from plain reductions (torch's dim=2 weight-norm kernels take
        ~0.45 ms each way on this [768, 48, 128] shape)."""
        p = self.conv.parametrizations.weight
        g, v = p.original0, p.original1
        return v * (g / v.pow(2).sum(dim=(0, 1), keepdim=True).sqrt())

    def add_to(self, x):
        """x + pos_conv(x) fused (HF/:689-690), the weight norm inside the op (Fn.PosConvWNFn)."""
        if os.environ.get("DFK_POSCONV_WN", "1") == "0":   # A/B: torch weight-norm ops + PosConvFn
            return Fn.PosConvFn.apply(x, self.weight(), self.conv.bias, self.groups)
        p = self.conv.parametrizations.weight
        return Fn.PosConvWNFn.apply(x, p.original0, p.original1, self.conv.bias, self.groups)


class Wav2Vec2Attention(nn.Module):
    """HF/:466-548: q/k/v/out projections; softmax(q k^T * hd^-0.5) v."""

    def __init__(self, embed_dim, num_heads, dropout=0.0):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.dropout = rng.Drop(dropout)
        self.head_dim = embed_dim // num_heads
        self.scaling = self.head_dim ** -0.5
        self.k_proj = nn.Linear(embed_dim, embed_dim)
        self.v_proj = nn.Linear(embed_dim, embed_dim)
        self.q_proj = nn.Linear(embed_dim, embed_dim)
        self.out_proj = nn.Linear(embed_dim, embed_dim)

    def flat_groups(self):
        """ParamStore adjacency: q/k/v weights and biases back to back -> one fused qkv GEMM operand."""
        q, k, v = self.q_proj, self.k_proj, self.v_proj
        return [[q.weight, k.weight, v.weight], [q.bias, k.bias, v.bias]]

    def core(self, x, B, T, skip=False):
        """x [B*T, C] -> attention output [B*T, C] before out_proj (skip=True: and an alias of x for the
        layer's residual, whose gradient joins the q/k/v dX GEMM)."""
        q, k, v = self.q_proj, self.k_proj, self.v_proj
        qkv = Fn.linear_group(x, (q.weight, k.weight, v.weight), (q.bias, k.bias, v.bias), skip=skip)
        if skip:
            qkv, xs = qkv
        geo = ((B, 1, 1, T), (1, 1, T), (1, 1, T), (0, 0, 0), self.num_heads, self.head_dim, self.scaling)
        d = self.dropout.spec() if self.dropout.active(self.training) else None
        out = Fn.window_attention(qkv, None, None, geo, drop=d)
        return (out, xs) if skip else out


class Wav2Vec2FeedForward(nn.Module):
    """HF/:551-573."""

    def __init__(self, config):
        super().__init__()
        self.intermediate_dense = nn.Linear(config.hidden_size, config.intermediate_size)
        self.output_dense = nn.Linear(config.intermediate_size, config.hidden_size)
        self.intermediate_dropout = rng.Drop(config.activation_dropout)
        self.output_dropout = rng.Drop(config.hidden_dropout)


class Wav2Vec2EncoderLayer(nn.Module):
    """HF/:575-608 (post-LN)."""

    def __init__(self, config):
        super().__init__()
        self.attention = Wav2Vec2Attention(config.hidden_size, config.num_attention_heads, config.attention_dropout)
        self.dropout = rng.Drop(config.hidden_dropout)
        self.layer_norm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.feed_forward = Wav2Vec2FeedForward(config)
        self.final_layer_norm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)

    def forward(self, x, B, T):
        tr = self.training
        ff = self.feed_forward
        spec = lambda d: d.spec() if d.active(tr) else None   # noqa: E731
        a, xs = self.attention.core(x, B, T, skip=True)
        x = Fn.layer_norm(Fn.linear(a, self.attention.out_proj.weight, self.attention.out_proj.bias, residual=xs,
                                    drop=spec(self.dropout)), self.layer_norm)
        x = Fn.mlp(x, ff.intermediate_dense, ff.output_dense, residual=x, drop_act=spec(ff.intermediate_dropout),
                   drop_out=spec(ff.output_dropout))
        return Fn.layer_norm(x, self.final_layer_norm)


class Wav2Vec2Encoder(nn.Module):
    """HF/:657-727 (no attention mask: equal-length clips, Q13)."""

    def __init__(self, config):
        super().__init__()
        if config.do_stable_layer_norm:
            raise NotImplementedError("stable-layer-norm encoder")
        self.pos_conv_embed = Wav2Vec2PositionalConvEmbedding(config)
        self.layer_norm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.dropout = rng.Drop(config.hidden_dropout)
        self.layers = nn.ModuleList([Wav2Vec2EncoderLayer(config) for _ in range(config.num_hidden_layers)])
        # LayerDrop coins: rank-independent draws (every replica drops the same layers, so the SGD skip of a
        # dropped layer's parameters stays identical across data-parallel ranks); 1 = run, 0 = skip
        self.layerdrop = rng.Drop(config.layerdrop, shared=True)
        self.register_buffer("layer_keep", torch.ones(config.num_hidden_layers), persistent=False)
        # OR of the coins since the last zero_grad (the SGD gate): with gradient accumulation a layer kept in
        # any micro-step of the window has a gradient in the reference (p.grad is not None) and is stepped
        self.register_buffer("layer_used", torch.zeros(config.num_hidden_layers), persistent=False)

    def param_gates(self):
        """(parameters, device flag) pairs for the fused SGD: a layer's parameters are stepped only when its
        LayerDrop coin kept it in some micro-step since the last zero_grad (training with layerdrop > 0)."""
        if self.layerdrop.p <= 0:
            return []
        return [(list(l.parameters()), self.layer_used[i:i + 1]) for i, l in enumerate(self.layers)]

    def reset_gates(self):
        """Called with zero_grad (ParamStore.zero_gates): a new accumulation window starts with no layer kept."""
        self.layer_used.zero_()

    def forward(self, h):
        B, T, C = h.shape
        d = self.dropout.spec() if self.dropout.active(self.training) else None
        x = Fn.layer_norm(self.pos_conv_embed.add_to(h.contiguous()), self.layer_norm, drop=d).reshape(B * T, C)
        lds = self.layerdrop.active(self.training)
        if lds:
            K.layerdrop_flags(self.layerdrop.spec(), self.layer_keep, self.layer_used)
        for i, layer in enumerate(self.layers):
            y = layer(x, B, T)
            if not lds:
                x = y
            elif x.is_cuda and y.dtype == x.dtype and (y.numel() * y.element_size()) % 16 == 0:
                x = Fn.LayerSelectFn.apply(y, x, self.layer_keep[i:i + 1])
            else:
                x = torch.where(self.layer_keep[i] > 0, y, x)
        return x.view(B, T, C)


class Wav2Vec2Model(nn.Module):
    """HF/:1244-1380 forward (SpecAugment / LayerDrop / dropouts must be off)."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.feature_extractor = Wav2Vec2FeatureEncoder(config)
        self.feature_projection = Wav2Vec2FeatureProjection(config)
        if config.mask_time_prob > 0.0 or config.mask_feature_prob > 0.0:
            self.masked_spec_embed = nn.Parameter(torch.empty(config.hidden_size).uniform_())
        self.encoder = Wav2Vec2Encoder(config)

        self.spec_site = rng.Drop(0.0)   # SpecAugment draws (site only)
        if config.mask_feature_prob > 0.0:
            raise NotImplementedError("SpecAugment feature masking (mask_feature_prob > 0)")

    def _mask_hidden_states(self, h):
        """HF/:1272-1317 time masking (training, apply_spec_augment, mask_time_prob > 0)."""
        c = self.config
        if not (self.training and c.apply_spec_augment and c.mask_time_prob > 0):
            return h
        return Fn.SpecAugmentFn.apply(h, self.masked_spec_embed, c.mask_time_prob, c.mask_time_length,
                                      c.mask_time_min_masks, self.spec_site.spec())

    def forward(self, input_values, attention_mask=None, **_):
        if attention_mask is not None:
            raise NotImplementedError("attention_mask (padded batches)")
        f = self.feature_extractor(input_values)
        h, ext = self.feature_projection(f)
        h = self._mask_hidden_states(h)
        return {"last_hidden_state": self.encoder(h), "extract_features": ext}
