"""Latency of the one-launch training BatchNorm (forward, + backward) by tensor size, inside a hipGraph of 20
calls (GPU-bound, no host gaps): where the per-launch floor sits and how it grows with rows / channels."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributed_examples_amd.ops import functional as OF  # noqa: E402

dev = torch.device("cuda")
shapes = [(64, 64), (128, 512), (512, 256), (512, 1024), (2048, 256), (8192, 64), (8192, 512), (32768, 64)]
for P, C in shapes:
    x = torch.randn(1, 1, P, C, device=dev).bfloat16()
    w = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev) * 0.1
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    res = {}
    for relu in (True,):
        def fwd():
            return OF.batch_norm(x, w, b, rm, rv, True, relu=relu)
        for _ in range(3):
            fwd()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.cuda.graph(g):
            for _ in range(20):
                fwd()
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res["fwd_us"] = round(e0.elapsed_time(e1) * 1e3 / 200, 2)
    stats = OF.bn_launch_stats()
    print(json.dumps({"P": P, "C": C, "MB": round(P * C * 2 / 1e6, 3), **res, "last_grid": stats.get("last_grid")}))
OF.check_device_errors("bn latency bench")
