import copy, os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from pytorch_distributed_examples_amd.models.resnet import ResNetShard2
from pytorch_distributed_examples_amd.ops import functional as OF
C = OF._C()
orig = OF._conv_backward
def wrapped(ctx, dy, x, weight, y=None):
    print("conv_backward dx_defer", getattr(ctx, "dx_defer", None), "grad_to", ctx.grad_to is not None, "join", ctx.join is not None, "geom", ctx.geom[:6], flush=True)
    r = orig(ctx, dy, x, weight, y)
    print("  pending after", C.pending_conv_count(), flush=True)
    return r
OF._conv_backward = wrapped
torch.manual_seed(5)
s2 = ResNetShard2()
blk = s2.seq[0][1]
b = copy.deepcopy(blk).cuda().train()
x = torch.randn(8, 8, 8, 1024).to(torch.bfloat16).cuda().requires_grad_()
y = b(x)
y.backward(torch.randn(y.shape).to(torch.bfloat16).cuda())
torch.cuda.synchronize()
print("slab uses", C.bn_bwd_slab_uses(), "pending", C.pending_conv_count())
