"""Inception-ResNet-v2 frame encoder on MI355X — drop-in for /root/reference/src/models/InceptionResV2.py
(class names, constructor signatures and state_dict keys kept).

Activations are channels-last [N, H, W, C] (one row of C channels per pixel), the layout every op here
consumes directly:
  Conv2d block (conv -> BatchNorm2d -> ReLU, :6-16)   dfk im2col2d + MFMA GEMM + dfk_bn2d (train / eval)
  1x1 stride-1 convs                                   the GEMM straight on the pixel rows (no im2col)
  MaxPool2d(3, 2) / AvgPool2d(3, 1, 1, no pad count)   dfk_pool2d
  residual blocks relu(x + scale * conv1x1(cat))      one GEMM with a bias / scale / residual / ReLU epilogue
  AdaptiveAvgPool2d((1, 1))                            dfk_rowmean over each frame's pixels
Branch outputs are concatenated along channels (torch.cat), as the reference.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import functional as Fn


def _pair(v):
    return tuple(v) if isinstance(v, (list, tuple)) else (v, v)


class Conv2d(nn.Module):
    """InceptionResV2.py:6-16 — Conv2d(bias) -> BatchNorm2d(eps=1e-3, momentum=0.1) -> ReLU."""

    def __init__(self, in_channels, out_channels, kernel_size, padding, stride=1, bias=True):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding, bias=bias)
        self.bn = nn.BatchNorm2d(out_channels, eps=0.001, momentum=0.1)
        self.relu = nn.ReLU(inplace=True)
        if bias:
            raise NotImplementedError("Conv2d block with a conv bias (the reference builds every one bias=False)")

    def forward(self, x):
        c = self.conv
        return Fn.ConvBNReLUFn.apply(x, c.weight, self.bn.weight, self.bn.bias, self.bn, _pair(c.kernel_size),
                                     _pair(c.stride), _pair(c.padding), self.training)


class _Pool(nn.Module):
    def __init__(self, mode, s, p):
        super().__init__()
        self.mode, self.s, self.p = mode, s, p

    def forward(self, x):
        return Fn.Pool2dFn.apply(x, 3, self.s, self.p, self.mode)


def _maxpool(stride):
    return _Pool(0, stride, 0)     # nn.MaxPool2d(3, stride=stride, padding=0)


def _seq(*mods):
    return nn.Sequential(*mods)


def _cat(xs):
    return torch.cat(xs, dim=-1)


class Reduction_A(nn.Module):
    """:19-35 (35 -> 17)."""

    def __init__(self, in_channels, k, l, m, n):
        super().__init__()
        self.branch_0 = Conv2d(in_channels, n, 3, stride=2, padding=0, bias=False)
        self.branch_1 = _seq(Conv2d(in_channels, k, 1, stride=1, padding=0, bias=False),
                             Conv2d(k, l, 3, stride=1, padding=1, bias=False),
                             Conv2d(l, m, 3, stride=2, padding=0, bias=False))
        self.branch_2 = _maxpool(2)

    def forward(self, x):
        return _cat((self.branch_0(x), self.branch_1(x), self.branch_2(x)))


class Stem(nn.Module):
    """:37-68."""

    def __init__(self, in_channels):
        super().__init__()
        self.features = _seq(Conv2d(in_channels, 32, 3, stride=2, padding=0, bias=False),
                             Conv2d(32, 32, 3, stride=1, padding=0, bias=False),
                             Conv2d(32, 64, 3, stride=1, padding=1, bias=False),
                             _maxpool(2),
                             Conv2d(64, 80, 1, stride=1, padding=0, bias=False),
                             Conv2d(80, 192, 3, stride=1, padding=0, bias=False),
                             _maxpool(2))
        self.branch_0 = Conv2d(192, 96, 1, stride=1, padding=0, bias=False)
        self.branch_1 = _seq(Conv2d(192, 48, 1, stride=1, padding=0, bias=False),
                             Conv2d(48, 64, 5, stride=1, padding=2, bias=False))
        self.branch_2 = _seq(Conv2d(192, 64, 1, stride=1, padding=0, bias=False),
                             Conv2d(64, 96, 3, stride=1, padding=1, bias=False),
                             Conv2d(96, 96, 3, stride=1, padding=1, bias=False))
        self.branch_3 = _seq(_Pool(1, 1, 1),    # nn.AvgPool2d(3, stride=1, padding=1, count_include_pad=False)
                             Conv2d(192, 64, 1, stride=1, padding=0, bias=False))

    def forward(self, x):
        x = self.features(x)
        return _cat((self.branch_0(x), self.branch_1(x), self.branch_2(x), self.branch_3(x)))


class _Residual(nn.Module):
    """relu?(x + scale * conv(cat(branches)))  (:90-95, :112-117, :159-166)."""

    def _res(self, x, branches, relu=True):
        return Fn.ResConvFn.apply(_cat(branches), self.conv.weight, self.conv.bias, x, self.scale, relu)


class Inception_ResNet_A(_Residual):
    """:71-95."""

    def __init__(self, in_channels, scale=1.0):
        super().__init__()
        self.scale = scale
        self.branch_0 = Conv2d(in_channels, 32, 1, stride=1, padding=0, bias=False)
        self.branch_1 = _seq(Conv2d(in_channels, 32, 1, stride=1, padding=0, bias=False),
                             Conv2d(32, 32, 3, stride=1, padding=1, bias=False))
        self.branch_2 = _seq(Conv2d(in_channels, 32, 1, stride=1, padding=0, bias=False),
                             Conv2d(32, 48, 3, stride=1, padding=1, bias=False),
                             Conv2d(48, 64, 3, stride=1, padding=1, bias=False))
        self.conv = nn.Conv2d(128, 320, 1, stride=1, padding=0, bias=True)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self._res(x, (self.branch_0(x), self.branch_1(x), self.branch_2(x)))


class Inception_ResNet_B(_Residual):
    """:98-117."""

    def __init__(self, in_channels, scale=1.0):
        super().__init__()
        self.scale = scale
        self.branch_0 = Conv2d(in_channels, 192, 1, stride=1, padding=0, bias=False)
        self.branch_1 = _seq(Conv2d(in_channels, 128, 1, stride=1, padding=0, bias=False),
                             Conv2d(128, 160, (1, 7), stride=1, padding=(0, 3), bias=False),
                             Conv2d(160, 192, (7, 1), stride=1, padding=(3, 0), bias=False))
        self.conv = nn.Conv2d(384, 1088, 1, stride=1, padding=0, bias=True)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self._res(x, (self.branch_0(x), self.branch_1(x)))


class Reduciton_B(nn.Module):
    """:120-142 (the reference's spelling)."""

    def __init__(self, in_channels):
        super().__init__()
        self.branch_0 = _seq(Conv2d(in_channels, 256, 1, stride=1, padding=0, bias=False),
                             Conv2d(256, 384, 3, stride=2, padding=0, bias=False))
        self.branch_1 = _seq(Conv2d(in_channels, 256, 1, stride=1, padding=0, bias=False),
                             Conv2d(256, 288, 3, stride=2, padding=0, bias=False))
        self.branch_2 = _seq(Conv2d(in_channels, 256, 1, stride=1, padding=0, bias=False),
                             Conv2d(256, 288, 3, stride=1, padding=1, bias=False),
                             Conv2d(288, 320, 3, stride=2, padding=0, bias=False))
        self.branch_3 = _maxpool(2)

    def forward(self, x):
        return _cat((self.branch_0(x), self.branch_1(x), self.branch_2(x), self.branch_3(x)))


class Inception_ResNet_C(_Residual):
    """:145-166."""

    def __init__(self, in_channels, scale=1.0, activation=True):
        super().__init__()
        self.scale = scale
        self.activation = activation
        self.branch_0 = Conv2d(in_channels, 192, 1, stride=1, padding=0, bias=False)
        self.branch_1 = _seq(Conv2d(in_channels, 192, 1, stride=1, padding=0, bias=False),
                             Conv2d(192, 224, (1, 3), stride=1, padding=(0, 1), bias=False),
                             Conv2d(224, 256, (3, 1), stride=1, padding=(1, 0), bias=False))
        self.conv = nn.Conv2d(448, 2080, 1, stride=1, padding=0, bias=True)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self._res(x, (self.branch_0(x), self.branch_1(x)), relu=self.activation)


class Inception_ResNetv2(nn.Module):
    """:169-190; forward(x [N, C, H, W]) -> [N, 1536] fp32 (channels-last inside)."""

    def __init__(self, in_channels=3, k=256, l=256, m=384, n=384, dropout_rate=0.0):
        super().__init__()
        blocks = [Stem(in_channels)]
        blocks += [Inception_ResNet_A(320, 0.17) for _ in range(10)]
        blocks.append(Reduction_A(320, k, l, m, n))
        blocks += [Inception_ResNet_B(1088, 0.10) for _ in range(20)]
        blocks.append(Reduciton_B(1088))
        blocks += [Inception_ResNet_C(2080, 0.20) for _ in range(9)]
        blocks.append(Inception_ResNet_C(2080, activation=False))
        self.features = nn.Sequential(*blocks)
        self.conv = Conv2d(2080, 1536, 1, stride=1, padding=0, bias=False)
        self.global_average_pooling = nn.AdaptiveAvgPool2d((1, 1))
        self.drop = dropout_rate
        self.compute_dtype = torch.float32

    def forward_nhwc(self, x):
        """x [N, H, W, C] channels-last -> [N, 1536] fp32 (global average pool, then F.dropout(p=drop), which
        the reference applies in training and eval alike: :187)."""
        y = self.conv(self.features(x.to(self.compute_dtype).contiguous()))
        N, H, W, C = y.shape
        f = Fn.RowMeanFn.apply(y.reshape(N * H * W, C), N)
        return F.dropout(f, self.drop) if self.drop > 0 else f

    def forward(self, x):
        return self.forward_nhwc(x.permute(0, 2, 3, 1))
