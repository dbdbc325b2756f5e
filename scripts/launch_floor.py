"""Per-kernel cost of a chain of tiny dependent kernels inside one hipGraph replay (the 'boundary' floor):
ATen add_ on one element and a native tiny kernel (cast_rows_ones on a 1x8 tensor)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_examples_amd import _native  # noqa: E402

C = _native.C()
dev = torch.device("cuda", 0)
a = torch.zeros(1, device=dev)
x = torch.zeros(1, 8, device=dev)
o = torch.zeros(1, 16, dtype=torch.bfloat16, device=dev)
big = torch.zeros(64 << 20, device=dev)  # 256 MB: dirty-L2 variant


def chain(kind, n):
    for _ in range(n):
        if kind == "aten_add":
            a.add_(1.0)
        elif kind == "native_tiny":
            C.cast_rows_ones(x, o)
        elif kind == "aten_add_after_4MB_write":
            big[: 1 << 20].add_(1.0)


res = {}
for kind in ("aten_add", "native_tiny", "aten_add_after_4MB_write"):
    n = 200
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        chain(kind, 5)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        chain(kind, n)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(10):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    res[kind] = round(t0.elapsed_time(t1) * 1000 / (10 * n), 3)
print(json.dumps({"us_per_kernel_in_graph": res}))
