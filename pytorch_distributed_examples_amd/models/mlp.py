"""MNIST MLP of the elastic-DDP example (pytorch_elastic/mnist_ddp_elastic.py:133-159, used with
``hidden_layers=5, features=1024`` at :172: 6,062,090 parameters).

Same module / parameter names as the reference ``Model`` (``input_layer``, ``hidden_layers.{i}``,
``final_layer``) so its ``MODEL_STATE`` snapshots load unchanged.  On GPU every layer is one bf16 MFMA
GEMM with bias + ReLU fused in the epilogue; in backward each layer's dgrad GEMM applies the ReLU mask of
its producer in the epilogue (threshold_backward fused), the final layer emits fp32 logits for the fused
cross-entropy kernel.
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops import layers as L


class MLP(nn.Module):
    def __init__(self, hidden_layers: int = 1, features: int = 128, in_features: int = 784, classes: int = 10):
        super().__init__()
        self.input_layer = L.Linear(in_features, features, relu=True)
        self.hidden_layers = nn.ModuleList([L.Linear(features, features, relu=True) for _ in range(hidden_layers)])
        self.final_layer = L.Linear(features, classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.reshape(x.size(0), -1)
        h = self.input_layer(x, consumer_masks=True)
        for layer in self.hidden_layers:
            h = layer(h, consumer_masks=True, mask_input_grad=True)
        return self.final_layer(h, out_f32=True, mask_input_grad=True)


def reference_mlp() -> MLP:
    """The configuration trained by the reference (mnist_ddp_elastic.py:172)."""
    return MLP(hidden_layers=5, features=1024)
