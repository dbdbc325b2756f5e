"""conv -> BatchNorm(+ReLU) with and without the split-K slab deferral: every intermediate and gradient
compared (the deferral must change nothing beyond summation-order rounding)."""
import sys

import torch

sys.path.insert(0, ".")
from pytorch_distributed_examples_amd.ops import functional as OF  # noqa: E402


def run(defer, shape, co, k, stride, pad, relu):
    OF._DEFER_CONV[0] = defer
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    n, h, w, ci = shape
    x = torch.randn(n, h, w, ci, generator=g).bfloat16().to(dev).requires_grad_()
    wt = (torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5).to(dev).requires_grad_()
    gamma = (torch.rand(co, generator=g) + 0.5).to(dev).requires_grad_()
    beta = torch.randn(co, generator=g).to(dev).requires_grad_()
    rm, rv = torch.zeros(co, device=dev), torch.ones(co, device=dev)
    y = OF.conv2d(x, wt, None, stride, pad, bn_follows=True)
    z = OF.batch_norm(y, gamma, beta, rm, rv, True, 0.1, 1e-5, None, relu)
    up = torch.randn(z.shape, generator=g).to(dev)
    (z.float() * up).sum().backward()
    torch.cuda.synchronize()
    return {"y": y.detach().float().clone(), "z": z.detach().float().clone(), "rm": rm, "rv": rv,
            "dx": x.grad.float(), "dw": wt.grad, "dg": gamma.grad, "db": beta.grad}


def main():
    for shape, co, k, s, p in [((8, 32, 32, 128), 128, 3, 2, 1), ((8, 16, 16, 512), 256, 1, 1, 0),
                               ((8, 8, 8, 1024), 256, 1, 1, 0), ((8, 32, 32, 256), 128, 1, 1, 0)]:
        for relu in (True, False):
            a, b = run(False, shape, co, k, s, p, relu), run(True, shape, co, k, s, p, relu)
            msg = []
            for key in a:
                d = (a[key] - b[key]).abs()
                rel = (d.norm() / (a[key].norm() + 1e-12)).item()
                msg.append(f"{key}:rel={rel:.2e},max={d.max().item():.2e}")
            print(shape, co, k, s, "relu" if relu else "", " ".join(msg), flush=True)
    print("pending convs left:", OF._C().pending_conv_count())


if __name__ == "__main__":
    main()
