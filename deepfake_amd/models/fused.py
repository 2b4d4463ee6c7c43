"""Builders for the north-star fused model: video slot
SwinTransformer3D (+ mean pooling, VSTFeat), mel slot SwinTransformerV2
(use_feat), waveform slot Audio2D(wav2vec2), FusionModel head.

CONFIGS mirror BASELINE.json: C1 = tiny VST 2,2,2,2 / window 4x7x7 + reduced
mel SwinV2 + 2-layer wav2vec2 (8x112x112, 1 s); C2 = Swin-T 2,2,6,2 / window
8x7x7 + SwinV2 (128; 2,2,18,2) + wav2vec2-base (32x224x224, 4 s); C4 =
Swin-B video (fp8=True: MX-fp8 GEMMs in its stages 3-4); C5 = 64 frames + 10 s audio.
"""
import os
import types

import torch

from . import set_compute_dtype, set_fp8
from .audioTransformer import Audio2D
from .ModalFusion import FusionModel
from .swin_transformer2d import SwinTransformerV2
from .video_swin_transformer import SwinTransformer3D, VSTFeat
from .wav2vec2 import Wav2Vec2Config, Wav2Vec2Model

HERE = os.path.dirname(os.path.abspath(__file__))
W2V_CONFIG = os.path.join(HERE, "w2v_base_config.json")

_VST_T = dict(patch_size=(2, 4, 4), embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24],
              window_size=(8, 7, 7), drop_path_rate=0.0, patch_norm=True)
_VST_B = dict(patch_size=(2, 4, 4), embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32],
              window_size=(8, 7, 7), drop_path_rate=0.0, patch_norm=True)
_MEL_C2 = dict(num_classes=1, use_feat=True, embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32],
               window_size=7, drop_path_rate=0.0, pretrained_window_sizes=(16, 16, 16, 16))

CONFIGS = {
    "c1": dict(vst=dict(patch_size=(2, 4, 4), embed_dim=96, depths=[2, 2, 2, 2], num_heads=[3, 6, 12, 24],
                        window_size=(4, 7, 7), drop_path_rate=0.0, patch_norm=True),
               mel=dict(num_classes=1, use_feat=True, img_size=224, embed_dim=32, depths=[2, 2, 2, 2],
                        num_heads=[1, 2, 4, 8], window_size=7, drop_path_rate=0.0,
                        pretrained_window_sizes=(16, 16, 16, 16)),
               w2v_layers=2, video_dim=768, audio_dim=256, T=8, H=112, W=112, seconds=1, B=2),
    "c2": dict(vst=_VST_T, mel=_MEL_C2, w2v_layers=12, video_dim=768, audio_dim=1024, T=32, H=224, W=224,
               seconds=4, B=8),
    "c4": dict(vst=_VST_B, mel=_MEL_C2, w2v_layers=12, video_dim=1024, audio_dim=1024, T=32, H=224, W=224,
               seconds=4, B=8),
    "c5": dict(vst=dict(_VST_T, use_checkpoint=True), mel=_MEL_C2, w2v_layers=12, video_dim=768, audio_dim=1024, T=64, H=224, W=224,
               seconds=10, B=8),
}


def build_fused(cfg, args=None, w2v_config=W2V_CONFIG, compute_dtype=torch.float32, regularize=False, fp8=False):
    """The north-star fused model.  regularize=False (parity / default): every dropout, DropPath,
    SpecAugment and LayerDrop off (Q12).  regularize=True: the reference's training regularisers — VST
    drop_path_rate 0.2 (SwinTransformer3D default, video_swin_transformer.py:500), SwinV2 0.1
    (swin_transformer2d.py:506), the wav2vec2-base checkpoint config's dropouts / LayerDrop /
    mask_time_prob, Audio2D's dropout (args.swin_drop) and the head's (args.classify_drop)."""
    if isinstance(cfg, str):
        cfg = CONFIGS[cfg]
    d = 0.1 if regularize else 0.0   # config.py:30-31 defaults of --classify_drop / --swin_drop
    args = args or types.SimpleNamespace(soft=0.01, classify_drop=d, swin_drop=d)
    vkw, mkw = dict(cfg["vst"]), dict(cfg["mel"])
    if regularize:
        vkw["drop_path_rate"], mkw["drop_path_rate"] = 0.2, 0.1
    vst = SwinTransformer3D(**vkw)
    mel = SwinTransformerV2(**mkw)
    wcfg = Wav2Vec2Config.from_json_file(w2v_config, num_hidden_layers=cfg["w2v_layers"])
    if not regularize:
        wcfg = wcfg.deterministic()
    pa = Audio2D(args, Wav2Vec2Model(wcfg), num_classes=1, use_feat=True)
    m = FusionModel(args, VSTFeat(vst), mel, pa, out_dim=1, video_dim=cfg["video_dim"], audio_dim=cfg["audio_dim"],
                    paudio_dim=768)
    if fp8:   # C4: MX-fp8 video-trunk GEMMs (bf16 compute everywhere else)
        st = os.environ.get("DFK_FP8_STAGES")   # A/B knob: 0-based stages on MX-fp8, e.g. "2,3" (default) or "0,1,2,3"
        set_fp8(m, tuple(int(v) for v in st.split(",") if v.strip()) if st is not None else cfg.get("fp8_stages", (2, 3)))
    return set_compute_dtype(m, compute_dtype)


def build_model(args, compute_dtype=torch.float32):
    """train.py:29-49 model choice by --modality, with the north-star video slot:
      fused  -> FusionModel(VSTFeat(SwinTransformer3D), SwinTransformerV2(use_feat), Audio2D(wav2vec2))
      video  -> VideoClassifier (SwinTransformer3D + mean-pool Mlp head, video_swin_transformer.py:688-793)
      audio  -> SwinTransformerV2(num_classes=1, 128; 2,2,18,2) (train.py:35)
      paudio -> Audio2D(wav2vec2-base) (train.py:39-41)
    Shapes come from --config; regularisers follow --deterministic."""
    from .video_swin_transformer import VideoClassifier
    cfg = CONFIGS[getattr(args, "config", "c2")]
    reg = not getattr(args, "deterministic", False)
    if getattr(args, "video_encoder", "swin") == "inception":   # the reference's current video branch
        from .IResNet import InceptionVideoClassifier
        drop = args.swin_drop if reg else 0.0
        if args.modality == "video":          # train.py:32
            return set_compute_dtype(InceptionVideoClassifier(args, 1, drop_rate=drop), compute_dtype)
        if args.modality == "fused":          # train.py:42-46: video_dim = hidden_size 1024
            m = build_fused(cfg, args, compute_dtype=compute_dtype, regularize=reg)
            ve = InceptionVideoClassifier(args, 1, drop_rate=drop, use_feat=True)
            m.vExtract = ve
            m.video_projection = torch.nn.Linear(1024, m.video_projection.out_features)
            return set_compute_dtype(m, compute_dtype)
    if args.modality == "fused":
        return build_fused(cfg, args, compute_dtype=compute_dtype, regularize=reg)
    if args.modality == "video":
        vkw = dict(cfg["vst"], drop_path_rate=0.2 if reg else 0.0)
        return set_compute_dtype(VideoClassifier(args, SwinTransformer3D(**vkw), num_classes=1), compute_dtype)
    if args.modality == "audio":
        mkw = dict(cfg["mel"], use_feat=False, drop_path_rate=0.1 if reg else 0.0)
        return set_compute_dtype(SwinTransformerV2(**mkw), compute_dtype)
    if args.modality == "paudio":
        wcfg = Wav2Vec2Config.from_json_file(W2V_CONFIG, num_hidden_layers=cfg["w2v_layers"])
        if not reg:
            wcfg = wcfg.deterministic()
        return set_compute_dtype(Audio2D(args, Wav2Vec2Model(wcfg), num_classes=1), compute_dtype)
    raise ValueError(f"unknown modality {args.modality!r}")
