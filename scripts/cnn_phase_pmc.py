"""Diagnostic for rocprofv3 --pmc: launches the fused CNN training kernel once per phase prefix
(stop_after = 1..11), so the per-dispatch counters of consecutive prefixes difference into per-phase counts
(scripts/pmc_summary.py --phases)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_examples_amd.models.cnn import Net  # noqa: E402
from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN  # noqa: E402

dev = torch.device("cuda")
net = Net().to(dev).train()
f = FusedCNN(net)
B = 1024
x = torch.randn(B, 1, 28, 28, device=dev)
y = torch.randint(0, 10, (B,), device=dev)
f.forward_backward(x, y)
torch.cuda.synchronize()
for k in list(range(1, 12)) + [-1]:
    f.stop_after = k
    f.forward_backward(x, y)
    torch.cuda.synchronize()
print("phase prefixes launched")
