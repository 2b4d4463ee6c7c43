"""FusionModel — drop-in for /root/reference/src/models/ModalFusion.py:7-75.

The head runs on [B, <=1536] features: its Linear layers are the MFMA GEMM
(fp32, M = clips), the 3x3 modality attention, BatchNorm1d (per-rank batch
statistics, momentum 0.08) and sigmoid are latency-trivial torch ops.
Extractor features arrive as fp32 [B, dim] whatever the trunk compute dtype.
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import functional as Fn
from ..utils import Mlp


class FusionModel(nn.Module):
    def __init__(self, args, VideoExtractor, AudioExtractor, PAudioExtractor, out_dim=2, video_dim=1024,
                 audio_dim=1024, paudio_dim=768, common_dim=512):
        super().__init__()
        self.vExtract, self.aExtract, self.paExtract = VideoExtractor, AudioExtractor, PAudioExtractor
        self.soft = args.soft
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
        self.drop = nn.Dropout(args.classify_drop)
        self.out_act = nn.Sigmoid()
        self.last_logits = None

    @staticmethod
    def _lin(x, m):
        return Fn.linear(x.float().contiguous(), m.weight, m.bias)

    def head(self, v_x, a_x, pa_x):
        """ModalFusion.py:37-75 (Q11: softmax(q k^T) THEN * 512^-0.5)."""
        v_x, a_x, pa_x = self._lin(v_x, self.video_projection), self._lin(a_x, self.audio_projection), \
            self._lin(pa_x, self.paudio_projection)
        comb = torch.stack((v_x, a_x, pa_x), dim=1)                       # B 3 C
        B = comb.shape[0]
        flat = comb.reshape(B * 3, -1)
        q = self._lin(flat, self.queries).view(B, 3, -1)
        k = self._lin(flat, self.keys).view(B, 3, -1)
        v = self._lin(flat, self.values).view(B, 3, -1)
        att = F.softmax(torch.einsum("bqd,bkd->bqk", q, k), dim=-1) * self.scaling
        att = self.drop(att)
        out = torch.einsum("bal,blv->bav", att, v).reshape(B, -1)
        feat = self.norm(Fn.linear(out.contiguous(), self.attn_proj.weight))
        feat = self.drop(feat)
        z = self.classify(feat)
        # detached: holding the graph would pin AccumulateGrad nodes to this step's stream (breaks graph capture)
        self.last_logits = z.detach()
        return self.out_act(z.squeeze())

    parallel_branches = False    # set by the training runtime (TrainStep), which also joins the streams

    def branch_streams(self):
        if not hasattr(self, "_streams"):
            # A/B knob: HIP stream priorities of the video / mel / waveform branches, e.g. "-1,0,0" (lower = higher)
            pr = os.environ.get("DFK_BRANCH_PRIO")
            ps = [int(v) for v in pr.split(",")] if pr else [0, 0, 0]
            self._streams = [torch.cuda.Stream(priority=p) for p in ps]
        return self._streams

    def join_branches(self):
        """Make the current stream wait for every branch stream (after backward: the direct-mode
        weight gradients the branch kernels wrote into the flat buffer)."""
        if hasattr(self, "_streams"):
            cur = torch.cuda.current_stream()
            for s in self._streams:
                cur.wait_stream(s)

    def forward(self, feature: tuple):
        """ModalFusion.py:30-75.  The three extractors are independent until the head: with
        parallel_branches they run on three HIP streams (video / mel / waveform), so the small-M
        GEMMs of the mel and wav2vec2 trunks fill the CUs the HBM-bound video trunk leaves idle; the
        autograd engine runs each backward op on its forward op's stream, so backward overlaps too."""
        video_feat, audio_feat, paudio_feat = feature
        if not (self.parallel_branches and video_feat.is_cuda):
            return self.head(self.vExtract(video_feat), self.aExtract(audio_feat), self.paExtract(paudio_feat))
        cur = torch.cuda.current_stream()
        capturing = torch.cuda.is_current_stream_capturing()
        outs = []
        for s, ext, x in zip(self.branch_streams(), (self.vExtract, self.aExtract, self.paExtract), feature):
            s.wait_stream(cur)
            if not capturing:
                x.record_stream(s)
            with torch.cuda.stream(s):
                outs.append(ext(x))
        for s, o in zip(self._streams, outs):
            cur.wait_stream(s)
            if not capturing:
                o.record_stream(cur)
        return self.head(*outs)

    def cal_nce_loss(self, p_a, p_b):
        """ModalFusion.py:78-99 (unused by the reference's training; kept for the API)."""
        pos = torch.logsumexp(torch.einsum("bd,bd->b", p_a, p_b).unsqueeze(-1) / self.soft, 1)
        l12 = torch.logsumexp(torch.einsum("bd,cd->bc", p_a, p_b) / self.soft, 1) - pos
        l21 = torch.logsumexp(torch.einsum("bd,cd->bc", p_b, p_a) / self.soft, 1) - pos
        return l12.mean() + l21.mean()
