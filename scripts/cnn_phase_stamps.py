"""Diagnostic: per-phase time of the fused CNN kernel from in-kernel wall_clock64 stamps (100 MHz)."""
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
for _ in range(5):
    f.forward_backward(x, y)
nwg = B // 4
f.stamps = torch.zeros(nwg, 16, dtype=torch.long, device=dev)
f.forward_backward(x, y)
torch.cuda.synchronize()
st = f.stamps.cpu().double()
d = (st[:, 1:12] - st[:, 0:11]) / 100.0  # us
names = ["P0 load", "P1 conv1", "P2 conv2", "P3 fc1", "P4a fc2", "P4b loss", "P5 fc2bwd", "P6 fc1bwd",
         "P7a c2wgrad", "P7b c2dgrad", "P9 conv1wgrad"]
for i, n in enumerate(names):
    print(f"{n:14s} median {d[:, i].median().item():7.2f} us  max {d[:, i].max().item():7.2f} us")
print("P1 conv1 MFMA part (stamp 1 -> 13) median", ((st[:, 13] - st[:, 1]) / 100.0).median().item(), "us;",
      "fragment wait + stores (13 -> 2)", ((st[:, 2] - st[:, 13]) / 100.0).median().item(), "us")
print("P1 conv1 MFMA part by wave: 0 / 15 median",
      [round(((st[:, k] - st[:, 1]) / 100.0).median().item(), 2) for k in (13, 15)], "us")
print("P9 split: loads + MFMAs + partials (10 -> 14)", ((st[:, 14] - st[:, 10]) / 100.0).median().item(),
      "us; combine + stores (14 -> 11)", ((st[:, 11] - st[:, 14]) / 100.0).median().item(), "us")
print("total median", (st[:, 11] - st[:, 0]).median().item() / 100.0, "us")
print("span (first start -> last stamp)", (st[:, 11].max() - st[:, 0].min()).item() / 100.0, "us")
print("workgroup start spread (last - first stamp 0)", (st[:, 0].max() - st[:, 0].min()).item() / 100.0, "us")
print("drain span (first start -> last workgroup end, stores drained)",
      (st[:, 12].max() - st[:, 0].min()).item() / 100.0, "us")
# the same launch timed from the host around a single stream-ordered call (includes dispatch + end of kernel)
s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
f.stamps = None
ts = []
for _ in range(20):
    torch.cuda.synchronize()
    s_ev.record()
    f.forward_backward(x, y)
    e_ev.record()
    torch.cuda.synchronize()
    ts.append(s_ev.elapsed_time(e_ev) * 1000.0)
ts.sort()
print(f"host events around one forward_backward (train + reduce): median {ts[len(ts) // 2]:.1f} us  min {ts[0]:.1f} us")
