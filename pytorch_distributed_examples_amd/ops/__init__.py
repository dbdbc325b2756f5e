"""Ops layer: autograd functions over the gfx950 HIP kernels, nn layers and fused optimisers."""
from . import functional
from .functional import (batch_norm, conv2d, cross_entropy, dropout, embedding_bag_sum, flatten_nchw,
                         global_avg_pool_flat, linear, log_softmax, max_pool2d, mse_loss, nll_loss,
                         to_native_image)
from .layers import BatchNorm2d, Conv2d, Dropout, Dropout2d, EmbeddingBag, Linear, MaxPool2d
from .optim import FusedAdam, FusedAdamW, FusedSGD

__all__ = [
    "functional", "batch_norm", "conv2d", "cross_entropy", "dropout", "embedding_bag_sum", "flatten_nchw",
    "global_avg_pool_flat", "linear", "log_softmax", "max_pool2d", "mse_loss", "nll_loss", "to_native_image",
    "BatchNorm2d", "Conv2d", "Dropout", "Dropout2d", "EmbeddingBag", "Linear", "MaxPool2d",
    "FusedAdam", "FusedAdamW", "FusedSGD",
]
