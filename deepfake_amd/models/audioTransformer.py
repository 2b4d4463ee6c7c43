"""Audio2D — drop-in for /root/reference/src/models/audioTransformer.py:5-30."""
import torch.nn as nn
import torch.nn.functional as F

from .. import functional as Fn
from ..utils import Mlp


class Audio2D(nn.Module):
    """wav_model(x).last_hidden_state -> mean over frames (AdaptiveAvgPool2d((1,in_feat)))
    -> F.dropout(p=args.swin_drop) — always on, as the reference (Q9) -> [B, in_feat]
    fp32 (use_feat=True); or the classifier branch (use_feat=False)."""

    def __init__(self, args, wav_model, in_feat=768, num_classes=2, use_feat=False):
        super().__init__()
        self.wav_model = wav_model
        self.use_feat = use_feat
        self.classifier = nn.Linear(512, num_classes)   # Q10: exists (unused) when use_feat=True
        self.model_drop = args.swin_drop
        if not use_feat:
            self.mlp = Mlp(in_feat, 512, 512)
            self.norm = nn.LayerNorm(512)
            self.act = nn.GELU()
            self.classify_drop = args.classify_drop

    def forward(self, x, mask=None):
        h = self.wav_model(x)["last_hidden_state"]
        B, T, C = h.shape
        feat = Fn.RowMeanFn.apply(h.reshape(B * T, C), B)
        if self.model_drop > 0:
            feat = F.dropout(feat, self.model_drop)
        if not self.use_feat:
            c = self.act(self.norm(self.mlp(feat)))
            if self.classify_drop > 0:
                c = F.dropout(c, self.classify_drop)
            return self.classifier(c).squeeze().sigmoid()
        return feat
