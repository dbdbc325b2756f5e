"""nn.Module layers over :mod:`.functional`.

Parameter / buffer names and initialisation match ``torch.nn`` (``weight``, ``bias``, ``running_mean``,
``running_var``, ``num_batches_tracked``) so model ``state_dict``s have the same keys and shapes as the
reference models built from ``torch.nn`` (e.g. the MLP of pytorch_elastic/mnist_ddp_elastic.py:133-159,
the CNN of horovod/mnist_horovod.py:9-25, ResNet-50 of rpc/model_parallel_ResNet50.py:43-139).
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import functional as OF


class Linear(nn.Module):
    """y = relu?(x W^T + b); fused on GPU (bias + ReLU in the MFMA GEMM epilogue)."""

    def __init__(self, in_features, out_features, bias=True, relu=False):
        super().__init__()
        self.in_features, self.out_features, self.relu = in_features, out_features, relu
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.weight._pde_linear = True  # the fused optimizer maintains its bf16 compute copy
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):  # == nn.Linear.reset_parameters
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(self.in_features) if self.in_features > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x, out_f32=False, consumer_masks=False, mask_input_grad=False):
        return OF.linear(x, self.weight, self.bias, self.relu, out_f32, consumer_masks, mask_input_grad)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, relu={self.relu}"


class Conv2d(nn.Module):
    """2-D convolution; NHWC implicit-GEMM on MFMA for GPU tensors."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True, relu=False):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding, self.relu = kernel_size, stride, padding, relu
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, kernel_size, kernel_size))
        self.weight._pde_conv = True  # the fused optimizer maintains its implicit-GEMM compute copies
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):  # == nn.Conv2d.reset_parameters
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in = self.in_channels * self.kernel_size * self.kernel_size
            bound = 1 / math.sqrt(fan_in)
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x, grad_join=None, grad_to=None, bn_follows=False, bn_stats=None, dx_bn=False):
        return OF.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.relu, grad_join, grad_to,
                         bn_follows, bn_stats, dx_bn)

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, stride={self.stride}, "
                f"padding={self.padding}, bias={self.bias is not None}")


class BatchNorm2d(nn.Module):
    """BatchNorm2d with optional fused (residual add, ReLU): relu?(bn(x) + residual)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        self._nbt_pending = 0

    def _flush_nbt(self):
        # GPU path counts batches on the host and folds them into the buffer lazily: one less kernel
        # launch per BN layer per step, same state_dict value.
        if self._nbt_pending:
            self.num_batches_tracked.add_(self._nbt_pending)
            self._nbt_pending = 0

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        self._flush_nbt()
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def forward(self, x, residual=None, relu=False, residual_grad_to=None):
        if self.training:
            n = OF.current_bn_groups()  # grouped BatchNorm: one tracked batch per micro-batch, as separately
            if x.is_cuda:
                self._nbt_pending += n
            else:
                self.num_batches_tracked.add_(n)
        return OF.batch_norm(x, self.weight, self.bias, self.running_mean, self.running_var, self.training,
                             self.momentum, self.eps, residual, relu, residual_grad_to)


class MaxPool2d(nn.Module):
    def __init__(self, kernel_size, stride=None, padding=0, relu=False):
        super().__init__()
        self.kernel_size, self.stride, self.padding, self.relu = kernel_size, stride or kernel_size, padding, relu

    def forward(self, x):
        return OF.max_pool2d(x, self.kernel_size, self.stride, self.padding, self.relu)


class Dropout(nn.Module):
    def __init__(self, p=0.5, channel=False):
        super().__init__()
        self.p, self.channel = p, channel

    def forward(self, x):
        return OF.dropout(x, self.p, self.training, self.channel)


class Dropout2d(Dropout):
    def __init__(self, p=0.5):
        super().__init__(p, channel=True)


class EmbeddingBag(nn.Module):
    """EmbeddingBag(mode='sum') with a wave-per-bag gather kernel and a scatter-add backward."""

    def __init__(self, num_embeddings, embedding_dim, mode="sum"):
        super().__init__()
        assert mode == "sum", "only mode='sum' (the reference's configuration) is implemented"
        self.num_embeddings, self.embedding_dim, self.mode = num_embeddings, embedding_dim, mode
        self.weight = nn.Parameter(torch.randn(num_embeddings, embedding_dim))

    def forward(self, indices, offsets):
        return OF.embedding_bag_sum(self.weight, indices, offsets)
