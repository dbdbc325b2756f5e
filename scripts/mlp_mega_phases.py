#!/usr/bin/env python3
"""Per-phase time of the one-launch MLP step (workgroup 0's wall-clock stamps, medians over steps)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_examples_amd.models.mlp import reference_mlp  # noqa: E402
from pytorch_distributed_examples_amd.models.mlp_mega import MegaMLP  # noqa: E402
from pytorch_distributed_examples_amd.ops.optim import FusedAdam  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = reference_mlp().to(dev)
    opt = FusedAdam(m.parameters(), lr=1e-3)
    mega = MegaMLP(m, opt)
    mega.stamps = torch.zeros(128, dtype=torch.int64, device=dev)
    x = torch.rand(128, 784, device=dev)
    y = torch.randint(0, 10, (128,), device=dev)
    rows = {}
    for i in range(40):
        mega.step(x, y)
        torch.cuda.synchronize()
        if i >= 10:
            for n, us, late in mega.phase_us():
                rows.setdefault(n, []).append((us, late))
    tot = totl = 0.0
    print(f"{'phase':22s} {'wg0 us':>8s} {'latest':>8s}")
    for n, v in rows.items():
        med = statistics.median(x[0] for x in v)
        late = statistics.median(x[1] for x in v)
        tot += med
        totl += late
        print(f"{n:22s} {med:8.2f} {late:8.2f}")
    print(f"{'sum':22s} {tot:8.2f} {totl:8.2f}   errors={mega.errors()}")


if __name__ == "__main__":
    main()
