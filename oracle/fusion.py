"""Oracle: FusionModel head and the composed north-star fused model (fp32 CPU).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates
/root/reference/src/models/ModalFusion.py:7-75 and the north-star composition
of SURVEY.md §0 (video slot SwinTransformer3D + mean, mel slot SwinV2
use_feat, waveform slot Audio2D(wav2vec2)).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import vst as V
from . import swinv2 as S2
from . import w2v as W
from .vst import Mlp


class FusionModel(nn.Module):
    """ModalFusion.py:7-75.  Q11: softmax(q k^T) THEN * 512^-0.5; BatchNorm1d(768,
    momentum 0.08); output sigmoid(z.squeeze())."""
    def __init__(self, v, a, pa, out_dim=1, video_dim=1024, audio_dim=1024, paudio_dim=768, common_dim=512,
                 classify_drop=0.0):
        super().__init__()
        self.vExtract, self.aExtract, self.paExtract = v, a, pa
        self.video_projection = nn.Linear(video_dim, common_dim)
        self.audio_projection = nn.Linear(audio_dim, common_dim)
        self.paudio_projection = nn.Linear(paudio_dim, common_dim)
        self.keys = nn.Linear(common_dim, common_dim)
        self.queries = nn.Linear(common_dim, common_dim)
        self.values = nn.Linear(common_dim, common_dim)
        self.scaling = common_dim ** -0.5
        self.attn_proj = nn.Linear(common_dim * 3, 768, bias=False)
        self.norm = nn.BatchNorm1d(768, momentum=0.08)
        self.classify = Mlp(768, 256, out_dim)
        self.drop = classify_drop
        self.last_logits = None

    def head(self, fv, fa, fp):
        x = torch.stack((self.video_projection(fv), self.audio_projection(fa), self.paudio_projection(fp)), 1)
        q, k, v = self.queries(x), self.keys(x), self.values(x)
        att = torch.softmax(torch.einsum("bqd,bkd->bqk", q, k), -1) * self.scaling
        att = F.dropout(att, self.drop, self.training)
        feat = torch.einsum("bal,blv->bav", att, v).flatten(1)
        feat = F.dropout(self.norm(self.attn_proj(feat)), self.drop, self.training)
        z = self.classify(feat)
        self.last_logits = z
        return torch.sigmoid(z.squeeze())

    def forward(self, feature):
        video, mel, wave = feature
        return self.head(self.vExtract(video), self.aExtract(mel), self.paExtract(wave))


def build_fused(cfg, w2v_config_json):
    """The fused model of tests/golden/golden_cases.py FUSED_C1-style configs."""
    vst = V.SwinTransformer3D(**cfg["vst"])
    mel = S2.SwinTransformerV2(**cfg["mel"])
    c = W.W2VConfig(w2v_config_json, num_hidden_layers=cfg["w2v_layers"], mask_time_prob=0.0)
    pa = W.Audio2D(W.Wav2Vec2Model(c))
    return FusionModel(V.VSTFeat(vst), mel, pa, out_dim=1, video_dim=cfg["video_dim"], audio_dim=cfg["audio_dim"])
