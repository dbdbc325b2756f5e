"""Time the K <= 128 forward GEMMs of ResNet-50 b32 (C.linear_fwd = the 1x1 conv GEMM) with CUDA events: the
low-K streamed kernel (default) or, under PDE_GEMM_LOWK=0, the 64x64 tile core.  One JSON line per shape:
us per launch and effective HBM bandwidth (A + B read, C written, bf16)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributed_examples_amd.ops import functional as OF  # noqa: E402

C = OF._C()
dev = torch.device("cuda")
shapes = [(32768, 64, 256), (8192, 128, 512), (32768, 64, 64), (32768, 128, 256), (8192, 64, 256)]
for M, K, N in shapes:
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.1).bfloat16()
    for _ in range(5):
        C.linear_fwd(x, w, None, False, False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 200
    e0.record()
    for _ in range(it):
        C.linear_fwd(x, w, None, False, False)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / it
    mb = 2 * (M * K + N * K + M * N) / 1e6
    print(json.dumps({"shape": f"{M}x{N}x{K}", "lowk": os.environ.get("PDE_GEMM_LOWK", "1") != "0",
                      "blocks_cap": os.environ.get("PDE_GEMM_LOWK_BLOCKS", "512"), "us": round(us, 2),
                      "TB_s": round(mb / us, 3)}))
# reference: what a pure write / copy of the largest output achieves on this box
y = torch.empty(32768, 256, device=dev, dtype=torch.bfloat16)
src = torch.empty_like(y)
for name, fn in (("fill 16 MB", lambda: y.fill_(1.0)), ("copy 16 MB", lambda: y.copy_(src))):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 200
    mb = 16.777 * (2 if name.startswith("copy") else 1)
    print(json.dumps({"shape": name, "us": round(us, 2), "TB_s": round(mb / us, 3)}))
