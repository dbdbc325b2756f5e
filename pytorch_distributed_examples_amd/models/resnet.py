"""ResNet-50 split into the two pipeline stages of rpc/model_parallel_ResNet50.py.

* :class:`Bottleneck` is implemented here (the reference imports torchvision's, :23; torchvision is not
  available -- SURVEY.md H7).  Same submodule names as torchvision (``conv1/bn1/conv2/bn2/conv3/bn3/
  downsample``), v1.5 layout (stride on the 3x3 conv).
* :class:`ResNetShard1` = stem conv7x7/s2 + BN + ReLU + maxpool3/s2 + layer1 + layer2
  (model_parallel_ResNet50.py:85-114; Kaiming-normal conv init, BN gamma=1/beta=0).
  :class:`ResNetShard2` = layer3 + layer4 + avgpool + fc (:117-139; default init, quirk Q11 kept).
  ``seq`` indices match the reference so ``state_dict`` keys are identical.
* GPU forward is NHWC bf16: every conv is an MFMA implicit-GEMM, every BatchNorm is the fused
  batch-statistics kernel with the ReLU -- and in the last BN of a block the residual add -- folded in.
  Activations stay on the device between stages (quirk Q13 fixed: no ``.cpu()`` hops).
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops import functional as OF
from ..ops import layers as L

EXPANSION = 4


class _ShapeOnly:
    """A stand-in carrying only ``.shape`` for shape-only planning (ops.functional.bn_fold_plan)."""

    def __init__(self, shape):
        self.shape = shape


class Bottleneck(nn.Module):
    expansion = EXPANSION

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = L.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = L.BatchNorm2d(width)
        self.conv2 = L.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = L.BatchNorm2d(width)
        self.conv3 = L.Conv2d(width, planes * EXPANSION, 1, bias=False)
        self.bn3 = L.BatchNorm2d(planes * EXPANSION)
        self.downsample = downsample
        self.stride = stride

    def _fold_plan(self, x):
        """(bn1 folded into conv2, bn2 folded into conv3) for this input shape / micro-batch grouping."""
        key = (tuple(x.shape), OF.current_bn_groups())
        plans = self.__dict__.setdefault("_pde_fold_plan", {})
        if key not in plans:
            c, w = self.conv1, self.conv2
            f1 = w.stride == 1 and OF.bn_fold_plan(x, c.in_channels, c.out_channels, 1, 1, 0, w.out_channels, 3, 1, 1)
            # the bn2 plan needs conv2's input shape only (= conv1's output: 1x1, stride 1)
            f2 = OF.bn_fold_plan(_ShapeOnly((x.shape[0], x.shape[1], x.shape[2], OF.pad8(w.in_channels))),
                                 w.in_channels, w.out_channels, 3, w.stride, 1, self.conv3.out_channels, 1, 1, 0)
            plans[key] = (f1, f2)
        return plans[key]

    def forward(self, x):
        identity = x
        # on the GPU x's two gradients (residual / downsample branch and conv1 branch) meet in conv1's dgrad
        # epilogue instead of an autograd add (ops.functional.GradJoin)
        join = OF.GradJoin() if (x.is_cuda and torch.is_grad_enabled() and x.requires_grad) else None
        t = self.training  # training-mode BatchNorm reduces a split-K conv's slabs itself (bn_follows)
        f1 = f2 = False
        if t and x.is_cuda and OF.bn_fold_enabled():
            # BatchNorm folded into the convolutions: the producer conv's epilogue emits the statistics, the
            # consumer conv applies bn + ReLU in its A loader (no BatchNorm launch in between)
            f1, f2 = self._fold_plan(x)
        g = OF.current_bn_groups()
        st2 = OF.BnFoldStats(self.bn2, g) if f2 else None
        if f1:
            st1 = OF.BnFoldStats(self.bn1, g)
            a1 = self.conv1(x, grad_join=join, bn_stats=st1)
            a2 = OF.bn_relu_conv(a1, st1, self.conv2, stats_out=st2, bn_follows=t)
        else:
            out = self.bn1(self.conv1(x, grad_join=join, bn_follows=t), relu=True)
            # bn1's output feeds conv2 alone (and bn2's conv3): their dgrads' split-K slabs go to the BatchNorm
            # backward unreduced (dx_bn)
            a2 = self.conv2(out, bn_follows=t, bn_stats=st2, dx_bn=t)
        if f2:
            out = OF.bn_relu_conv(a2, st2, self.conv3, bn_follows=t)
        else:
            out = self.conv3(self.bn2(a2, relu=True), bn_follows=t, dx_bn=t)
        if self.downsample is not None:
            conv, bn = self.downsample[0], self.downsample[1]
            identity = bn(conv(x, grad_to=join, bn_follows=t))
        # relu(bn3(conv3(.)) + identity) in one fused kernel
        return self.bn3(out, residual=identity, relu=True, residual_grad_to=join if self.downsample is None else None)


class _StemReLU(nn.Module):
    """Placeholder at seq[2] (the reference's nn.ReLU): the ReLU is fused into seq[1]'s BatchNorm."""

    def forward(self, x):  # pragma: no cover - never called on its own
        return torch.relu(x)


def make_layer(inplanes, planes, blocks, stride=1):
    downsample = None
    if stride != 1 or inplanes != planes * EXPANSION:
        downsample = nn.Sequential(L.Conv2d(inplanes, planes * EXPANSION, 1, stride=stride, bias=False),
                                   L.BatchNorm2d(planes * EXPANSION))
    layers = [Bottleneck(inplanes, planes, stride, downsample)]
    for _ in range(1, blocks):
        layers.append(Bottleneck(planes * EXPANSION, planes))
    return nn.Sequential(*layers)


class ResNetShard1(nn.Module):
    """Stage 1: [N,3,H,W] fp32 NCHW -> [N,16,16,512] (GPU, NHWC bf16) / [N,512,16,16] (CPU) at 128x128."""

    def __init__(self, device=None):
        super().__init__()
        self.seq = nn.Sequential(
            L.Conv2d(3, 64, 7, stride=2, padding=3, bias=False),
            L.BatchNorm2d(64),
            _StemReLU(),
            L.MaxPool2d(3, 2, 1),
            make_layer(64, 64, 3),
            make_layer(256, 128, 4, stride=2),
        )
        for m in self.modules():
            if isinstance(m, L.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, L.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if device is not None:
            self.to(device)

    def forward(self, x):
        if x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.shape[1] == 3:
            x = OF.to_native_image(x)
        s = self.seq
        x = s[1](s[0](x, bn_follows=self.training), relu=True)
        x = s[3](x)
        return s[5](s[4](x))


class ResNetShard2(nn.Module):
    """Stage 2: layer3 + layer4 + avgpool + fc -> [N, 1000] fp32 logits."""

    def __init__(self, device=None, num_classes=1000):
        super().__init__()
        self.seq = nn.Sequential(
            make_layer(512, 256, 6, stride=2),
            make_layer(1024, 512, 3, stride=2),
            nn.AdaptiveAvgPool2d((1, 1)),
        )
        self.fc = L.Linear(512 * EXPANSION, num_classes)
        if device is not None:
            self.to(device)

    def forward(self, x):
        x = self.seq[1](self.seq[0](x))
        x = OF.global_avg_pool_flat(x)
        return self.fc(x, out_f32=True)


class ResNet50(nn.Module):
    """Both stages on one device (single-GPU / pure data-parallel configuration)."""

    def __init__(self, device=None, num_classes=1000):
        super().__init__()
        self.shard1 = ResNetShard1()
        self.shard2 = ResNetShard2(num_classes=num_classes)
        if device is not None:
            self.to(device)

    def forward(self, x):
        return self.shard2(self.shard1(x))
