"""Case definitions shared by the golden generator and the parity tests.

Pure data: no reference import.  Weights for every case are re-created with
oracle.fill.named_fill_(seed), inputs with oracle.fill.randn(seed+k, shape).
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# copied config.json values we need live in w2v_config.json next to this file
W2V_CONFIG_JSON = os.path.join(HERE, "w2v_config.json")

# WindowAttention3D (video_swin_transformer.py:91-173)
WATTN_CASES = [
    # shifted window, N=196, with compute_mask over a 4x14x14 volume (nW = 4)
    dict(name="wattn_n196_mask", dim=64, heads=2, full_window=(4, 7, 7), N=196, B_=4,
         mask_dhw=(4, 14, 14), shift=(2, 3, 3), seed=11),
    # N=392 (Swin-T 8x7x7), unshifted, 3 heads of 32
    dict(name="wattn_n392", dim=96, heads=3, full_window=(8, 7, 7), N=392, B_=2, seed=21),
    # Q3: clamped window 4x4x4 (N=64) indexing the full 4x7x7 RPB table
    dict(name="wattn_n64_clamped", dim=64, heads=2, full_window=(4, 7, 7), N=64, B_=2, seed=31),
]

# SwinTransformerBlock3D (:176-278)
BLOCK_CASES = [
    dict(name="block_shift", dim=64, heads=2, window=(4, 7, 7), shift=(2, 3, 3), shape=(1, 4, 14, 14), seed=41),
    dict(name="block_noshift", dim=64, heads=2, window=(4, 7, 7), shift=(0, 0, 0), shape=(1, 4, 14, 14), seed=51),
    # padded H/W (10 -> 14), shifted: exercises pad-after-LN and the mask over padded volume
    dict(name="block_pad_shift", dim=64, heads=2, window=(4, 7, 7), shift=(2, 3, 3), shape=(1, 4, 10, 10), seed=61),
    # clamped D (2 <= 4 -> window 2, shift 0 along D), shift only along H/W
    dict(name="block_clampD", dim=64, heads=2, window=(4, 7, 7), shift=(2, 3, 3), shape=(2, 2, 14, 14), seed=71),
]

PATCH_EMBED = dict(name="patch_embed", patch=(2, 4, 4), dim=96, shape=(2, 3, 8, 32, 32), seed=81)
MERGE_CASES = [
    dict(name="merge_even", dim=64, shape=(1, 4, 14, 14, 64), seed=91),
    dict(name="merge_odd", dim=64, shape=(1, 2, 7, 7, 64), seed=101),
]

VST_C1 = dict(name="vst_c1", seed=111, shape=(1, 3, 8, 112, 112),
              kwargs=dict(patch_size=(2, 4, 4), embed_dim=96, depths=[2, 2, 2, 2], num_heads=[3, 6, 12, 24],
                          window_size=(4, 7, 7), drop_path_rate=0.0, patch_norm=True))


def w2v_overrides(layers):
    """Deterministic wav2vec2 (Q12): every dropout, LayerDrop and SpecAugment off."""
    return dict(num_hidden_layers=layers, hidden_dropout=0.0, attention_dropout=0.0, activation_dropout=0.0,
                feat_proj_dropout=0.0, layerdrop=0.0, mask_time_prob=0.0, final_dropout=0.0,
                hidden_dropout_prob=0.0)


W2V_C1 = dict(name="w2v_2layer_1s", layers=2, B=1, seconds=1, seed=121)
W2V_GRAD_KEYS = ("conv_layers.0.conv.weight", "conv_layers.0.layer_norm", "conv_layers.3.conv.weight",
                 "feature_projection", "pos_conv_embed", "layers.0.attention.q_proj", "layers.1.feed_forward",
                 "encoder.layer_norm", "layers.1.final_layer_norm")

HEAD = dict(name="fusion_head", B=4, video_dim=768, audio_dim=256, seed=131)

FUSED_C1 = dict(
    name="fused_c1", seed=141, B=2, T=8, H=112, W=112, seconds=1, lr=0.01, wd=0.05,
    vst=VST_C1["kwargs"],
    mel=dict(num_classes=1, use_feat=True, img_size=224, embed_dim=32, depths=[2, 2, 2, 2], num_heads=[1, 2, 4, 8],
             window_size=7, drop_path_rate=0.0, pretrained_window_sizes=(16, 16, 16, 16)),
    w2v_layers=2, video_dim=768, audio_dim=256)


# ---------------------------------------------------------------- C2 shapes
# Swin-T stage-1 SW-MSA block over a whole C2 clip's stage-1 volume: N=392 windows, shift (4,3,3)
BLOCK_C2_S1 = dict(name="block_c2_s1", dim=96, heads=3, window=(8, 7, 7), shift=(4, 3, 3), shape=(1, 16, 56, 56),
                   seed=151)
# stage 4: H=W=7 <= window -> get_window_size keeps only the D shift (4,0,0) (Q6); 2 windows along D
BLOCK_C2_S4 = dict(name="block_c2_s4", dim=768, heads=24, window=(8, 7, 7), shift=(4, 3, 3), shape=(1, 16, 7, 7),
                   seed=161)
# C4 (Swin-B video trunk, BASELINE configs[3]): stage 1 (dim 128, 4 heads, N=392, shift 4x3x3, a whole clip's
# 16x56x56 volume) and stage 3 (dim 512, 16 heads, 16x14x14: 8 windows, shift 4x3x3) — the bf16 and MX-fp8 blocks
BLOCK_C4_S1 = dict(name="block_c4_s1", dim=128, heads=4, window=(8, 7, 7), shift=(4, 3, 3), shape=(1, 16, 56, 56),
                   seed=191)
BLOCK_C4_S3 = dict(name="block_c4_s3", dim=512, heads=16, window=(8, 7, 7), shift=(4, 3, 3), shape=(1, 16, 14, 14),
                   seed=195)
# SwinV2-B mel stage 3 (C2 mel branch): 14x14 tokens, C=512, 16 heads, window 7, blocks shift 0 / 3,
# pretrained_window_size 16 (the CPB-MLP coordinate normalisation), two clips
MEL_C2_S3 = dict(name="mel_c2_s3", dim=512, heads=16, res=(14, 14), window=7, pretrained=16, B=2, seed=171)

FUSED_C2 = dict(
    name="fused_c2", seed=181, B=2, T=32, H=224, W=224, seconds=4, lr=0.01, wd=0.05,
    vst=dict(patch_size=(2, 4, 4), embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24],
             window_size=(8, 7, 7), drop_path_rate=0.0, patch_norm=True),
    mel=dict(num_classes=1, use_feat=True, embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32],
             window_size=7, drop_path_rate=0.0, pretrained_window_sizes=(16, 16, 16, 16)),
    w2v_layers=12, video_dim=768, audio_dim=1024)

# the reference's Inception-ResNet-v2 + NeXtVLAD video branch, smallest viable frame size
INCEPTION = dict(name="inception_b2t2", seed=191, B=2, T=2, HW=75, sample=256,
                 bn_keys=("inceptionRes.features.0.features.0.bn.running_mean",
                          "inceptionRes.features.0.features.0.bn.running_var",
                          "inceptionRes.features.5.branch_1.1.bn.running_var",
                          "inceptionRes.conv.bn.running_mean", "video_nextvlad.bn0.running_mean",
                          "video_nextvlad.bn1.running_var", "bn0.running_mean", "bn1.running_var"))

GRAD_SAMPLE_C1 = 1024   # per-parameter gradient tensors of the fused train steps: strided samples + norm
GRAD_SAMPLE_C2 = 512


def fixture_compress(key, a, big=65536, sample=8192):
    """Tensors above ``big`` elements are stored as key@sub (every step-th
    element of the flat array, about ``sample`` of them), key@sum and key@norm (float64)."""
    import numpy as np
    a = np.asarray(a)
    if a.size <= big:
        return {key: a}
    step = -(-a.size // sample)
    f = a.reshape(-1).astype(np.float64)
    return {key + "@sub": a.reshape(-1)[::step].copy(), key + "@step": np.array(step),
            key + "@shape": np.array(a.shape), key + "@sum": np.array(f.sum()),
            key + "@norm": np.array(np.sqrt((f * f).sum()))}


# ---------------------------------------------------------------- f2: PIL frame transform fixtures
PIL_FRAMES = dict(name="pil_frames", seed=201)


def pil_test_image(seed, h, w, channels=3):
    """Deterministic decoded-frame stand-in (uint8 [h, w, channels]): smooth gradients and blobs with noise, so
    the antialiased resize sees real structure at every scale (regenerated by the tests, never stored)."""
    import numpy as np
    g = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    out = np.empty((h, w, channels), dtype=np.uint8)
    for c in range(channels):
        fx, fy, ph = g.uniform(2, 40), g.uniform(2, 40), g.uniform(0, 6.28)
        v = 128 + 60 * np.sin(2 * np.pi * x / w * fx + ph) * np.cos(2 * np.pi * y / h * fy) + 40 * (x / w - y / h)
        v += g.normal(0, 12, size=(h, w))
        out[..., c] = np.clip(np.rint(v), 0, 255).astype(np.uint8)
    return out[..., 0] if channels == 1 else out


# ---------------------------------------------------------------- pretrained-weight loaders
PRETRAINED = dict(name="pretrained", seed=211,
                  vst=dict(patch_size=(2, 4, 4), embed_dim=96, depths=[2, 2, 2, 2], num_heads=[3, 6, 12, 24],
                           window_size=(4, 7, 7), patch_norm=True),
                  mel=dict(num_classes=1, use_feat=True, img_size=224, embed_dim=32, depths=[2, 2, 2, 2],
                           num_heads=[1, 2, 4, 8], window_size=7, pretrained_window_sizes=(16, 16, 16, 16)))


def synth_swin2d_checkpoint(shapes, seed):
    """A 2-D Swin checkpoint {'model': state_dict} for a 3-D model with the given {key: shape}: every key with the
    2-D shape — patch_embed.proj.weight without the patch-depth axis, relative_position_bias_table [(2*12-1)^2, nH]
    (a window-12 pretraining: bicubic-resized on load) in stages 0-1 and [(2*7-1)^2, nH] in stages 2-3 — plus
    entries the loader must drop (relative_position_index, attn_mask) and one it must ignore (head.weight)."""
    import torch
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for k, shp in shapes.items():
        if k == "patch_embed.proj.weight":
            shp = (shp[0], shp[1], shp[3], shp[4])
        elif "relative_position_bias_table" in k:
            side = 23 if k.startswith(("layers.0.", "layers.1.")) else 13
            shp = (side * side, shp[1])
        elif "relative_position_index" in k:
            sd[k] = torch.zeros(169, 169, dtype=torch.long)
            continue
        sd[k] = torch.randn(shp, generator=g) * 0.02
    sd["layers.0.blocks.1.attn_mask"] = torch.full((4, 49, 49), -100.0)
    sd["head.weight"] = torch.randn(10, 768, generator=g)
    return {"model": sd}


def synth_swinv2_checkpoint(shapes, seed):
    """{'checkpoint': state_dict} for a SwinV2 model: every parameter random, and the re-initialised buffers
    (relative_coords_table, relative_position_index) filled with garbage the loader must drop."""
    import torch
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for k, shp in shapes.items():
        if "relative_position_index" in k:
            sd[k] = torch.zeros(shp, dtype=torch.long)
        elif "relative_coords_table" in k:
            sd[k] = torch.full(shp, 7.0)
        else:
            sd[k] = torch.randn(shp, generator=g) * 0.05
    return {"checkpoint": sd}
