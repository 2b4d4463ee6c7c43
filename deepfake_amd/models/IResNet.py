"""InceptionVideoClassifier + NeXtVLAD — drop-in for /root/reference/src/models/IResNet.py:247-393, the video
branch the reference's train.py:45 trains.  The frame encoder is the HIP
Inception-ResNet-v2 (InceptionResV2.py); NeXtVLAD and the gated head run on [B, T, 1536] features, with their
Linear layers on the dfk GEMM and the small BatchNorm1d / softmax / sigmoid / normalize steps as stock ops
(latency-bound, < 0.1 % of the branch's FLOPs).  State_dict keys match the reference's.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import functional as Fn
from .InceptionResV2 import Inception_ResNetv2


def _lin(x, m):
    shp = x.shape
    return Fn.linear(x.float().reshape(-1, shp[-1]).contiguous(), m.weight, m.bias).view(*shp[:-1], m.weight.shape[0])


class NeXtVLAD(nn.Module):
    """IResNet.py:247-329."""

    def __init__(self, dim=1024, num_clusters=64, lamb=2, groups=8, max_frames=300, bn_mom=0.1):
        super().__init__()
        self.num_clusters, self.dim, self.alpha, self.bn_mom = num_clusters, dim, 0, bn_mom
        self.K, self.G = num_clusters, groups
        self.group_size = int((lamb * dim) // self.G)
        self.fc0 = nn.Linear(dim, lamb * dim)
        self.fc_gk = nn.Linear(lamb * dim, self.G * self.K)
        self.fc_g = nn.Linear(lamb * dim, self.G)
        self.cluster_weights2 = nn.Parameter(torch.rand(1, self.group_size, self.K))
        self.bn0 = nn.BatchNorm1d(max_frames, momentum=self.bn_mom)
        self.bn1 = nn.BatchNorm1d(1, momentum=self.bn_mom)

    def forward(self, x, mask=None):
        _, M, N = x.shape
        x_dot = _lin(x, self.fc0)                                            # B M λN
        x_tilde = x_dot.reshape(-1, M, self.G, self.group_size)
        wgk = self.bn0(_lin(x_dot, self.fc_gk)).reshape(-1, M * self.G, self.K)
        alpha_gk = F.softmax(wgk, dim=-1)
        alpha_g = torch.sigmoid(_lin(x_dot, self.fc_g))
        if mask is not None:
            alpha_g = alpha_g * mask.unsqueeze(2)
        activation = alpha_gk * alpha_g.reshape(-1, M * self.G, 1)             # B (MG) K
        a = activation.sum(-2, keepdim=True) * self.cluster_weights2          # B (λN/G) K
        vlad = torch.matmul(activation.permute(0, 2, 1), x_tilde.reshape(-1, M * self.G, self.group_size))
        vlad = F.normalize(vlad.permute(0, 2, 1) - a, 1)
        vlad = self.bn1(vlad.reshape(-1, 1, self.K * self.group_size))
        return vlad.reshape(-1, self.K * self.group_size)


class InceptionVideoClassifier(nn.Module):
    """IResNet.py:331-393; forward(x [B, T, C, H, W]) -> probabilities [B] (or features [B, hidden] with
    use_feat).  The frames enter the encoder channels-last ([B*T, H, W, C]) without the reference's
    rearrange copy to [B*T, C, H, W]."""

    def __init__(self, args, num_classes, in_channels=3, num_clusters=64, lamb=2, hidden_size=1024, groups=8,
                 max_frames=300, drop_rate=0.5, gating_reduction=8, pretrained_resnet=None, use_feat=False):
        super().__init__()
        self.inceptionRes = Inception_ResNetv2(in_channels=3, dropout_rate=drop_rate)   # dim = 1536
        dim = 1536
        self.bn_mom = args.bn_momentum
        self.use_feat = use_feat
        self.drop_rate = drop_rate
        self.group_size = int((lamb * dim) // groups)
        self.fc0 = nn.Linear(num_clusters * self.group_size, hidden_size)
        self.bn0 = nn.BatchNorm1d(1, momentum=self.bn_mom)
        self.fc1 = nn.Linear(hidden_size, hidden_size // gating_reduction)
        self.bn1 = nn.BatchNorm1d(1, momentum=self.bn_mom)
        self.fc2 = nn.Linear(hidden_size // gating_reduction, hidden_size)
        if not use_feat:
            self.logistic = nn.Linear(hidden_size, num_classes)
            self.classify_drop = nn.Dropout(args.classify_drop)
        self.video_nextvlad = NeXtVLAD(dim, max_frames=args.num_frames, lamb=lamb, num_clusters=num_clusters,
                                       groups=groups, bn_mom=self.bn_mom)

    def forward(self, x, mask=None):
        b, t, c, h, w = x.shape
        f = self.inceptionRes.forward_nhwc(x.permute(0, 1, 3, 4, 2).reshape(b * t, h, w, c))
        vlad = self.video_nextvlad(f.view(b, t, -1), mask=mask)
        if self.drop_rate > 0.:
            vlad = F.dropout(vlad, p=self.drop_rate)     # always on, as the reference (:374)
        activation = F.relu(self.bn0(_lin(vlad, self.fc0).unsqueeze(1)).squeeze())
        gates = self.bn1(_lin(activation, self.fc1).unsqueeze(1)).squeeze()
        feat = activation * torch.sigmoid(_lin(gates, self.fc2))
        if not self.use_feat:
            return torch.sigmoid(self.classify_drop(_lin(feat, self.logistic).squeeze()))
        return feat
