"""Fused multi-tensor optimisers: SGD, Adam, AdamW.

GPU parameters are updated by ONE ``multi_tensor_optim`` launch per param group (csrc/kernels/optim.hip)
whose hyper-parameters and step counter live in device memory, so the update is hipGraph-capturable
and an LR change between replays (Horovod-elastic ``on_state_reset``, horovod_mnist_elastic.py:80-82)
is honoured.  The same launch refreshes the bf16 compute copies of the weights it updates (linear and
1x1-conv weights, whose compute layout is a plain cast), so those layers never re-derive them per step
(:func:`.functional.maintain_compute_copies`).  CPU parameters use the same math in plain torch (the
reference's CPU configuration).

The per-parameter state uses torch's key names (``step``, ``exp_avg``, ``exp_avg_sq``,
``momentum_buffer``) so ``state_dict()`` round-trips with ``torch.optim`` and with the elastic
``TorchState`` commit/restore.
"""
from __future__ import annotations

import torch

from .. import _native
from . import functional as OF
from . import streams

_MODES = {"sgd": 0, "adam": 1, "adamw": 2}


class _FusedBase(torch.optim.Optimizer):
    KIND = "adam"

    def __init__(self, params, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, momentum=0.0,
                 grad_scale=1.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, momentum=momentum,
                        grad_scale=grad_scale)
        super().__init__(params, defaults)
        self._dev = {}  # id(group) -> dict(table, sig, hp, hp_key, step)

    # -- GPU -----------------------------------------------------------------------------------
    def _group_dev(self, gi, group, params):
        C = _native.C()
        st = self._dev.get(gi)
        dev = params[0].device
        if st is None:
            st = {"sig": None, "hp_key": None,
                  "hp": torch.zeros(8, dtype=torch.float32, device=dev),
                  # {steps taken, arrival counter of the update kernel}
                  "step": torch.zeros(2, dtype=torch.int32, device=dev)}
            # a new group state (new optimizer, or after load_state_dict): the host step is authoritative once
            s0 = self.state[params[0]].get("step") if params else None
            st["step"][0].fill_(int(s0) if s0 is not None else 0)
            self._dev[gi] = st
        need_avg = self.KIND in ("adam", "adamw") or group["momentum"] != 0.0
        for p in params:
            state = self.state[p]
            if self.KIND in ("adam", "adamw"):
                if "exp_avg" not in state:
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            elif need_avg and "momentum_buffer" not in state:
                state["momentum_buffer"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
        grads = [p.grad for p in params]
        if self.KIND in ("adam", "adamw"):
            m = [self.state[p]["exp_avg"] for p in params]
            v = [self.state[p]["exp_avg_sq"] for p in params]
        else:
            m = [self.state[p]["momentum_buffer"] for p in params] if need_avg else []
            v = []
        sig = tuple((p.data_ptr(), g.data_ptr(), g.is_contiguous()) for p, g in zip(params, grads)) + \
            tuple(t.data_ptr() for t in m) + tuple(t.data_ptr() for t in v)
        if st["sig"] != sig:
            # (re)build the tables; the device step counter carries on
            grads_c = [g if g.is_contiguous() else g.contiguous() for g in grads]
            copies = [OF.maintain_compute_copies(p) or {} for p in params]
            none = torch.empty(0, device=params[0].device)
            bf = [c.get("bf16", none) for c in copies]
            table, chunks, nchunks = C.optim_table([p.data for p in params], grads_c, m, v, bf)
            st.update(sig=sig, table=table, chunks=chunks, nchunks=nchunks, grads_keep=grads_c)
            # KxK conv weights: both bf16 GEMM layouts refreshed by one launch after the update
            kxk = [(p, c) for p, c in zip(params, copies) if "kxk" in c]
            st["conv_table"], st["nconv"], st["conv_blocks"] = None, 0, 0
            if kxk:
                st["conv_table"] = C.conv_layout_table([p.data for p, _ in kxk], [c["conv_fwd"] for _, c in kxk],
                                                       [c["conv_dgrad"] for _, c in kxk],
                                                       [c["kxk"][0] for _, c in kxk], [c["kxk"][1] for _, c in kxk])
                st["nconv"] = len(kxk)
                # x blocks per entry: the largest weight's 32x32 (co, ci) tiles (3x3 path) / 256-pair chunks
                tiles = max(-(-c["kxk"][0] // 32) * -(-c["kxk"][1] // 32) for _, c in kxk)
                st["conv_blocks"] = max(1, min(1024, tiles))
        b1, b2 = group["betas"]
        hp_key = (group["lr"], b1, b2, group["eps"], group["weight_decay"], group["momentum"], group["grad_scale"])
        if st["hp_key"] != hp_key:
            st["hp"].copy_(torch.tensor(list(hp_key) + [0.0], dtype=torch.float32), non_blocking=False)
            st["hp_key"] = hp_key
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        C = None
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            if params[0].is_cuda:
                C = C or _native.C()
                streams.join(params[0].device)  # gradients written on the wgrad side stream
                st = self._group_dev(gi, group, params)
                C.optim_step(st["table"], st["chunks"], st["nchunks"], _MODES[self.KIND], st["hp"], st["step"])
                if st["nconv"]:
                    C.conv_layouts_step(st["conv_table"], st["nconv"], st["conv_blocks"])
                # host ``step`` is synchronised from the device counter by state_dict() (graph replays)
            else:
                self._cpu_step(group, params)
        OF.bump_weight_generation()
        return loss

    # -- update segments: one layer's update appended to a later backward GEMM launch ------------
    def _segment(self, subset):
        """(table, chunks, c0, c1, mode, hp, step) of ``subset`` -- parameters contiguous in the (single, GPU)
        param group's order -- for ``optim_attach`` / ``optim_step_range``."""
        assert len(self.param_groups) == 1, "update segments: one parameter group"
        group = self.param_groups[0]
        params = [p for p in group["params"] if p.grad is not None]
        st = self._group_dev(0, group, params)
        chunk = _native.C().optim_chunk_elems()
        starts, c = {}, 0
        for p in params:
            starts[id(p)] = c
            c += -(-p.numel() // chunk)
        ids = [id(p) for p in subset]
        c0 = min(starts[i] for i in ids)
        c1 = max(starts[id(p)] + -(-p.numel() // chunk) for p in subset)
        assert c1 - c0 == sum(-(-p.numel() // chunk) for p in subset), "segment parameters must be contiguous"
        return st["table"], st["chunks"], c0, c1, _MODES[self.KIND], st["hp"], st["step"]

    def supports_segments(self, params) -> bool:
        """True when :meth:`attach_update` / :meth:`step_range` can run this optimiser's update piecewise:
        one GPU parameter group, no KxK conv layout copies to refresh."""
        # (inspects the maintained copies without re-allocating them: maintain_compute_copies would replace the
        # copies the optimiser table writes)
        return (len(self.param_groups) == 1 and all(p.is_cuda for p in params) and
                not any(getattr(p, "_pde_conv", False) and p.dim() == 4 and p.shape[2] * p.shape[3] > 1
                        for p in params) and
                not any("kxk" in p.__dict__.get("_pde_maint", {}) for p in params))

    @torch.no_grad()
    def attach_update(self, subset):
        """Append the update of ``subset`` (whose gradients are final) to the NEXT paired backward GEMM launch
        as extra blocks (``OF.gemm_pair``): the HBM-bound update overlaps the latency-bound GEMMs."""
        t, ch, c0, c1, mode, hp, step = self._segment(subset)
        _native.C().optim_attach(t, ch, c0, c1, mode, hp, step, False)

    @torch.no_grad()
    def step_range(self, subset, last: bool = True):
        """The update of ``subset`` as its own launch; ``last``: the step's final segment (advances the device
        step counter -- every parameter must have been updated by a segment of this step)."""
        t, ch, c0, c1, mode, hp, step = self._segment(subset)
        _native.C().optim_step_range(t, ch, c0, c1, mode, hp, step, last)
        if last:
            OF.bump_weight_generation()

    # -- CPU reference math (torch.optim semantics) ---------------------------------------------
    def _cpu_step(self, group, params):
        lr, (b1, b2), eps = group["lr"], group["betas"], group["eps"]
        wd, mom, gs = group["weight_decay"], group["momentum"], group["grad_scale"]
        for p in params:
            g = p.grad if gs == 1.0 else p.grad * gs
            state = self.state[p]
            state["step"] = state.get("step", 0) + 1
            t = state["step"]
            if self.KIND == "sgd":
                if wd != 0:
                    g = g.add(p, alpha=wd)
                if mom != 0:
                    buf = state.get("momentum_buffer")
                    if buf is None or t == 1:
                        buf = g.clone()
                    else:
                        buf.mul_(mom).add_(g)
                    state["momentum_buffer"] = buf
                    g = buf
                p.add_(g, alpha=-lr)
                continue
            if self.KIND == "adamw":
                p.mul_(1 - lr * wd)
            elif wd != 0:
                g = g.add(p, alpha=wd)
            if "exp_avg" not in state:
                state["exp_avg"] = torch.zeros_like(p)
                state["exp_avg_sq"] = torch.zeros_like(p)
            m, v = state["exp_avg"], state["exp_avg_sq"]
            m.lerp_(g, 1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            bc1 = 1 - b1 ** t
            bc2 = 1 - b2 ** t
            denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
            p.addcdiv_(m, denom, value=-lr / bc1)

    def sync_step_from_device(self):
        """Copy each GPU group's device step counter into the per-parameter host ``step``.  The device counter
        is authoritative: hipGraph replays of a captured training step (and the fused CNN update kernels)
        advance it without running this Python code."""
        for gi, group in enumerate(self.param_groups):
            st = self._dev.get(gi)
            if st is None:
                continue
            steps = int(st["step"][0].item())
            for p in group["params"]:
                if p in self.state:
                    self.state[p]["step"] = steps

    def state_dict(self):
        self.sync_step_from_device()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dev = {}


class FusedSGD(_FusedBase):
    KIND = "sgd"

    def __init__(self, params, lr, momentum=0.0, weight_decay=0.0, grad_scale=1.0):
        super().__init__(params, lr=lr, momentum=momentum, weight_decay=weight_decay, grad_scale=grad_scale)


class FusedAdam(_FusedBase):
    KIND = "adam"

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, grad_scale=1.0):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, grad_scale=grad_scale)


class FusedAdamW(_FusedBase):
    KIND = "adamw"

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, grad_scale=1.0):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, grad_scale=grad_scale)
