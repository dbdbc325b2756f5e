"""Fused training step for the MNIST CNN (csrc/kernels/cnn_fused.hip).

:class:`FusedCNN` flattens a :class:`~.cnn.Net`'s parameters into ONE contiguous fp32 buffer in torch
parameter order (the ``nn.Parameter`` objects stay the same, their storage becomes views of the flat
buffer, so optimizers / ``state_dict`` / DDP keep working) and runs forward + NLL + backward of the
whole batch in one kernel launch plus one deterministic slab-reduction that writes the gradients
straight into a flat gradient buffer -- the DDP wrapper's, when it is laid out in forward order.

    fused = FusedCNN(net)
    ddp = DistributedDataParallel(net, overlap=False, param_order="forward")
    loss = fused.forward_backward(x, y, grad_out=ddp.flat_grad)   # grads written, no autograd
    ddp.sync_gradients(); opt.step()

Semantics match ``nll_loss(net(x), y)`` + ``backward()`` in train mode, including Dropout2d(p=0.5) on
conv2's output and dropout(p=0.5) on fc1's (fresh masks every call; dropout disabled in eval mode).

Fused optimiser step (plain SGD, the reference's ``optim.SGD(lr=0.01)``, mnist_horovod.py:50): the training
kernel reads the conv weights as a bf16 MFMA fragment image that a prep kernel writes from the fp32
parameters.  With ``sgd=opt`` (single process) the slab reduction also applies the SGD update and rewrites
the fragment slots of the weights it updates; with :meth:`sgd_step` (after the gradient all-reduce) one
kernel does the same.  Either way the next step skips the prep launch::

    loss = fused.forward_backward(x, y, grad_out=buf, sgd=opt)          # world 1: 2 launches per step
    loss = fused.forward_backward(x, y, grad_out=g, sgd=opt, xgmi=xa)   # world > 1 on one node: 2 launches
    loss = fused.forward_backward(x, y, grad_out=ddp.flat_grad)         # world > 1, any data plane:
    ddp.sync_gradients(); fused.sgd_step(opt, ddp.flat_grad)            #   3 launches + all-reduce

With ``xgmi`` (a :class:`..parallel.xgmi_allreduce.XgmiAllreduce` over the data-parallel ranks) the slab
reduction exchanges every workgroup's gradient chunk with all peers over xGMI inside the same kernel and
sums the ranks' chunks in rank order (``avg``: x 1/world), so ``grad_out`` receives the all-reduced
gradients, identical on every rank, and the SGD update stays fused -- the all-reduce costs no launch.

The fragment image is re-derived (prep launch) whenever anything other than these fused updates may have
written the weights: any other optimiser step bumps the weight generation (:func:`.functional.
bump_weight_generation`); direct writes (``load_state_dict``, broadcasts) must call :meth:`invalidate`.
"""
from __future__ import annotations

import torch

from .. import _native
from ..ops import functional as OF


class FusedCNN:
    def __init__(self, net, workgroups: int | None = None):
        C = _native.C()
        self.net = net
        self.params = list(net.parameters())
        n = sum(p.numel() for p in self.params)
        assert n == C.cnn_num_params(), f"not the reference Net ({n} params)"
        dev = self.params[0].device
        flat = torch.empty(n, dtype=torch.float32, device=dev)
        off = 0
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                flat[off:off + k].copy_(p.detach().reshape(-1))
                p.data = flat[off:off + k].view_as(p)
                off += k
        self.flat = flat
        OF.bump_weight_generation()  # parameter storage moved: drop cached compute copies
        self.own_grad = None
        self.workgroups = workgroups
        self.stamps = None  # diagnostic: int64 [nwg, 16] tensor of per-phase wall-clock stamps
        self.stop_after = -1  # diagnostic: end the training kernel after phase stamp k (counter attribution)
        self.frag = torch.empty(C.cnn_frag_bytes(), dtype=torch.uint8, device=dev)
        self._frag_gen = None  # weight generation at which the fragment image was last made current
        # an optimiser other than the fused SGD updates the weights every step (AdamW, hipGraph-replayed): the
        # kernel rebuilds its bf16 fragment image from the fp32 weights at every step (k_cnn_prep fused in)
        self.always_prep = False

    def invalidate(self):
        """The fp32 weights were written behind our back: rebuild the fragment image next step."""
        self._frag_gen = None

    @staticmethod
    def _sgd_hp(opt):
        """Device hyper-parameters of a FusedSGD that the fused update can apply (plain SGD only)."""
        from ..ops.optim import FusedSGD

        assert isinstance(opt, FusedSGD) and len(opt.param_groups) == 1, "fused update needs one FusedSGD group"
        group = opt.param_groups[0]
        assert group["momentum"] == 0.0 and group["weight_decay"] == 0.0, "fused update is plain SGD"
        params = [p for p in group["params"] if p.grad is not None]
        st = opt._group_dev(0, group, params)
        for p in params:  # the fused update writes the fp32 weights only (plus its own fragment image)
            OF.release_compute_copies(p)
        return (st["hp"], st["step"]), params

    def _after_update(self, opt, params):
        # the step count lives in the optimizer's device counter (advanced by the fused kernels, so hipGraph
        # replays count too); FusedSGD.state_dict() reads it back
        OF.bump_weight_generation()
        self._frag_gen = OF.weight_generation()

    @torch.no_grad()
    def sgd_step(self, opt, grads: torch.Tensor):
        """``opt.step()`` for the flat parameters (plain SGD) fused with the fragment-image refresh."""
        (hp, step), params = self._sgd_hp(opt)
        _native.C().cnn_sgd(self.flat, grads, hp, self.frag, step)
        self._after_update(opt, params)

    def _bind_adamw_state(self, opt):
        """The FusedAdamW's exp_avg / exp_avg_sq become views of two flat buffers (state_dict keeps working); a state
        tensor replaced behind our back (load_state_dict of an elastic restore) is copied in and re-bound."""
        if getattr(self, "_adam_m", None) is None:
            self._adam_m = torch.zeros_like(self.flat)
            self._adam_v = torch.zeros_like(self.flat)
        off = 0
        for p in self.params:
            k = p.numel()
            st = opt.state[p]
            for key, flat in (("exp_avg", self._adam_m), ("exp_avg_sq", self._adam_v)):
                view = flat[off:off + k].view_as(p)
                cur = st.get(key)
                if cur is None or cur.data_ptr() != view.data_ptr():
                    with torch.no_grad():
                        if cur is None:
                            view.zero_()
                        else:
                            view.copy_(cur.reshape(p.shape))
                    st[key] = view
            off += k

    @torch.no_grad()
    def adamw_step(self, opt, grads: torch.Tensor):
        """``opt.step()`` of a one-group FusedAdamW over the flat parameters fused with the fragment-image refresh:
        ONE launch (``k_cnn_adamw``) instead of the multi-tensor update plus the next step's prep launch; the update
        math and the device step counter are the optimiser's own (optim_device.h)."""
        from ..ops.optim import FusedAdamW

        assert isinstance(opt, FusedAdamW) and len(opt.param_groups) == 1, "adamw_step needs one FusedAdamW group"
        self._bind_adamw_state(opt)
        group = opt.param_groups[0]
        params = [p for p in group["params"] if p.grad is not None]
        st = opt._group_dev(0, group, params)
        _native.C().cnn_adamw(self.flat, grads, self._adam_m, self._adam_v, st["hp"], self.frag, st["step"])
        OF.bump_weight_generation()
        self._frag_gen = OF.weight_generation()

    def _nwg(self, B: int) -> int:
        if self.workgroups:
            return self.workgroups
        # ~4 images per workgroup, one workgroup per CU (256 CUs); 2 fit per CU by LDS
        return max(1, min(512, (B + 3) // 4))

    def grad_buffer(self) -> torch.Tensor:
        """A flat gradient buffer whose views are installed as ``p.grad`` (when no DDP buffer is used)."""
        if self.own_grad is None:
            self.own_grad = torch.zeros_like(self.flat)
            off = 0
            for p in self.params:
                k = p.numel()
                p.grad = self.own_grad[off:off + k].view_as(p)
                off += k
        return self.own_grad

    def forward_backward(self, x: torch.Tensor, y: torch.Tensor, grad_out: torch.Tensor | None = None,
                         accumulate: bool = False, p_drop2: float = 0.5, p_drop1: float = 0.5,
                         sgd=None, xgmi=None, avg: bool = True) -> torch.Tensor:
        """Loss (device scalar) of the local batch; gradients of the mean loss written to ``grad_out``.

        ``sgd``: a plain FusedSGD over these parameters -- also take the optimiser step.
        ``xgmi``: an XgmiAllreduce over the data-parallel ranks -- ``grad_out`` receives the all-reduced
        gradients (``avg``: averaged), exchanged inside the reduction kernel."""
        C = _native.C()
        if grad_out is None:
            grad_out = self.grad_buffer()
        x = x.float().contiguous()
        y = y.long().contiguous()
        training = self.net.training
        prep = self.always_prep or self._frag_gen is None or self._frag_gen != OF.weight_generation()
        (hp, step), params = self._sgd_hp(sgd) if sgd is not None else ((None, None), None)
        view, xscale = None, 1.0
        if xgmi is not None and xgmi.size > 1:
            view, xscale = xgmi.view(), (1.0 / xgmi.size if avg else 1.0)
        loss = C.cnn_train(x, y, self.flat, OF._rng_counter(x.device), p_drop2, p_drop1, training, grad_out,
                           accumulate, None, self.stamps, self.frag, prep, hp, self.stop_after, step, view, xscale)
        if sgd is not None:
            self._after_update(sgd, params)
        else:
            # the weights did not change: the image stays current until someone writes them
            self._frag_gen = OF.weight_generation()
        return loss
