"""MNIST CNN ``Net`` of the Horovod examples (horovod/mnist_horovod.py:9-25 ==
horovod/horovod_mnist_elastic.py:16-32; 21,840 parameters).

conv(1->10,k5) -> maxpool2 -> ReLU -> conv(10->20,k5) -> Dropout2d -> maxpool2 -> ReLU -> view(320)
-> fc(320->50) -> ReLU -> dropout -> fc(50->10) -> log_softmax(dim=1)

Parameter names match the reference (``conv1``, ``conv2``, ``fc1``, ``fc2``).  The reference calls
``F.log_softmax`` without ``dim`` (implicit dim=1, deprecated: SURVEY.md Q9); we pass ``dim=1``.

GPU path: NHWC bf16 with channels zero-padded to multiples of 8 (1->8, 10->16, 20->24), implicit-GEMM
convs on MFMA, maxpool fused with the following ReLU, channel dropout on the conv2 output, fp32 logits.
A whole-network fused kernel path (``fused=True``) is in :mod:`.cnn_fused`.
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops import functional as OF
from ..ops import layers as L


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = L.Conv2d(1, 10, kernel_size=5)
        self.conv2 = L.Conv2d(10, 20, kernel_size=5)
        self.conv2_drop = L.Dropout2d()
        self.fc1 = L.Linear(320, 50, relu=True)
        self.fc2 = L.Linear(50, 10)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = OF.to_native_image(x)
        x = OF.max_pool2d(self.conv1(x), 2, relu=True)
        x = OF.max_pool2d(self.conv2_drop(self.conv2(x)), 2, relu=True)
        x = OF.flatten_nchw(x, 20)
        x = self.fc1(x)
        x = OF.dropout(x, 0.5, self.training)
        x = self.fc2(x, out_f32=True)
        return OF.log_softmax(x, dim=1)
