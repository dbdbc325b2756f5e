"""The elastic-DDP MLP's whole training step as ONE persistent kernel launch (csrc/kernels/mlp_fused.hip).

Reference: pytorch_elastic/mnist_ddp_elastic.py:133-173 (``Model``: Linear + ReLU stack, ``CrossEntropyLoss``,
``optimizer.step()``); model of :mod:`.mlp`:

    mega = MegaMLP(model, opt)        # opt: FusedAdam / FusedAdamW / FusedSGD over model.parameters() (one group)
    loss = mega.step(x, y)            # forward + cross-entropy + backward + optimiser update: 1 launch

    mega = MegaMLP(model, opt, xgmi=MegaMLP.exchange(model, device))   # world > 1 on one node (collective)
    loss = mega.step(x, y)            # ... with DDP's gradient average INSIDE the same launch

World > 1 (single node): every 64x64 weight-gradient tile is exchanged with the other ranks over xGMI between its
GEMM and its update, inside the launch (csrc/kernels/mlp_fused.hip ``xchg_tile``: staged into this rank's IPC slot,
one flag per workgroup and exchange, summed over the ranks in rank order, x 1/world) -- the gradients of layer j
cross the links while layer j-1's backward runs, and the step stays ONE launch at any world size.  Adam / AdamW
(the fused update form) only.

Forward, loss, backward and the update of every layer run phase after phase inside one grid of one workgroup per
CU (grid barriers between phases), each phase one global round trip.  The results are those of the layer-by-layer
path (:class:`.mlp_fused.FusedMLP` + ``opt.step()``): same bf16 operands, fp32 accumulation, the optimiser's own
per-element update (optim_device.h); gradients land in ``p.grad``, the optimiser state in ``opt.state``, the device
step counter advances, and the bf16 weight copies the layers read are refreshed -- an eager ``model(x)`` after the
step sees the updated weights.  ``kernel_launches_per_step() == 1``.

The grid barriers need every workgroup resident: ``step`` refuses to run while CUs are reserved for kernels spinning
on other streams (``bn_reserve_headroom``), and an eager caller's ``step`` reads the barrier error word every
``check_every`` calls (a device sync; graph replays are checked by :meth:`errors` at the caller's commit / epoch
boundary) and raises :class:`DeviceBarrierError` -- a timed-out barrier means the step's hand-offs raced.
"""
from __future__ import annotations

import os

import torch

from .. import _native
from ..ops import functional as OF
from ..ops.optim import _MODES


class DeviceBarrierError(RuntimeError):
    """A grid barrier of the one-launch MLP step timed out: not every workgroup was resident, the phase hand-offs
    raced and the weights / optimiser state written by that step are not trustworthy."""


class MegaMLP:
    @staticmethod
    def exchange(net, device, group=None, timeout_s: float | None = None):
        """The xGMI instance the in-launch exchange of ``net``'s gradient tiles needs (collective over ``group``)."""
        from ..parallel.xgmi_allreduce import XgmiAllreduce

        layers = [net.input_layer, *net.hidden_layers, net.final_layer]
        floats = sum(-(-L.out_features // 64) * -(-L.in_features // 64) * (64 * 64 + 64) for L in layers)
        grid = int(_native.C().mlp_train_grid())
        return XgmiAllreduce(device, group=group, max_bytes=floats * 4 + (1 << 20), blocks=max(grid, 1),
                             timeout_s=timeout_s, key=None)

    def __init__(self, net, opt, check_every: int = 64, xgmi=None):
        self.net, self.opt = net, opt
        self.layers = [net.input_layer, *net.hidden_layers, net.final_layer]
        for i, L in enumerate(self.layers):
            assert L.bias is not None and L.relu == (i < len(self.layers) - 1), "Linear+ReLU stack, plain last layer"
        assert len(opt.param_groups) == 1, "one optimiser parameter group"
        self.params = [p for L in self.layers for p in (L.weight, L.bias)]
        assert [id(p) for p in opt.param_groups[0]["params"]] == [id(p) for p in self.params], \
            "the optimiser must hold exactly the model's parameters, in model order"
        self.mode = _MODES[opt.KIND]
        self._bufs: dict = {}
        self._grid = None
        self.calls = 0
        self.check_every = int(check_every)
        self.xgmi = xgmi  # parallel.xgmi_allreduce.XgmiAllreduce: the in-launch gradient exchange (world > 1)
        if xgmi is not None and self.mode == 0:
            raise ValueError("MegaMLP: the in-launch gradient exchange needs Adam / AdamW (the fused update form)")
        self.stamps = None  # set to a zeroed int64[128] GPU tensor: phase-boundary clocks (100 MHz), see phase_us

    def _buffers(self, B: int, dev: torch.device):
        key = (B, str(dev))
        if key not in self._bufs:
            bf = dict(dtype=torch.bfloat16, device=dev)
            act, actT, d, dT = [], [], [], []
            for i, L in enumerate(self.layers):
                fin = L.in_features
                actT.append(torch.empty(fin, B, **bf))
                if i == 0:
                    act.append(torch.empty(0, **bf)); d.append(torch.empty(0, **bf)); dT.append(torch.empty(0, **bf))
                else:
                    act.append(torch.empty(B, fin, **bf))
                    d.append(torch.empty(B, fin, **bf))
                    dT.append(torch.empty(fin, B, **bf))
            self._bufs[key] = dict(
                act=act, actT=actT, d=d, dT=dT,
                dlog=torch.zeros(B, 32, **bf), dlogT=torch.zeros(32, B, **bf),  # zero padding is never written
                loss_part=torch.zeros(B // 32, dtype=torch.float32, device=dev),
                bar=torch.zeros(512, dtype=torch.int32, device=dev), err=torch.zeros(1, dtype=torch.int32, device=dev))
        return self._bufs[key]

    def grid(self) -> int:
        if self._grid is None:
            self._grid = int(_native.C().mlp_train_grid())
        return self._grid

    @torch.no_grad()
    def step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """One training step on (x [B, 784] fp32 images or [B, 1, 28, 28], y [B] labels); returns the mean loss."""
        C = _native.C()
        B = x.shape[0]
        if B % 32:
            raise ValueError(f"MegaMLP: batch {B} must be a multiple of 32")
        if C.bn_headroom_reserved() > 0:
            raise RuntimeError("MegaMLP: CUs are reserved for kernels spinning on other streams; the persistent grid "
                               "(one workgroup per CU) could not be co-resident -- use FusedMLP")
        capturing = torch.cuda.is_current_stream_capturing()
        if not capturing and self.check_every > 0 and self.calls and self.calls % self.check_every == 0:
            self.check()
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        group = self.opt.param_groups[0]
        st = self.opt._group_dev(0, group, self.params)  # state tensors, device hyper-parameters and step counter
        nl = len(self.layers)
        wbf, wtbf = [], []
        for i, L in enumerate(self.layers):
            wbf.append(OF._maintained(L.weight, "bf16"))
            wtbf.append(OF.maintain_transposed_copy(L.weight, 32 if i == nl - 1 else L.out_features) if i > 0
                        else torch.empty(0, dtype=torch.bfloat16, device=x.device))
        bufs = self._buffers(B, x.device)
        state = self.opt.state
        none = torch.empty(0, device=x.device)

        def st_of(p, key):
            return state[p].get(key, none)

        mkey = "exp_avg" if self.mode != 0 else "momentum_buffer"
        loss = torch.empty(1, dtype=torch.float32, device=x.device)
        C.mlp_train(x.reshape(B, -1).float().contiguous(), y.long().contiguous(),
                    [L.weight for L in self.layers], [L.bias for L in self.layers],
                    [L.weight.grad for L in self.layers], [L.bias.grad for L in self.layers],
                    [st_of(L.weight, mkey) for L in self.layers], [st_of(L.weight, "exp_avg_sq") for L in self.layers],
                    [st_of(L.bias, mkey) for L in self.layers], [st_of(L.bias, "exp_avg_sq") for L in self.layers],
                    wbf, wtbf, bufs["act"], bufs["actT"], bufs["d"], bufs["dT"], bufs["dlog"], bufs["dlogT"],
                    bufs["loss_part"], loss, st["hp"], st["step"], self.mode, bufs["bar"], bufs["err"], self.grid(),
                    self.stamps,
                    self.xgmi.view() if self.xgmi is not None else None,
                    1.0 / self.xgmi.size if self.xgmi is not None else 1.0)
        # the weights changed on the device: the in-place writes bypass the version counters, so stamp the
        # copies current (they were refreshed by the same kernel) and invalidate generation-keyed caches
        for L in self.layers:
            d = L.weight.__dict__.get("_pde_maint")
            if d is not None:
                d["version"] = L.weight._version
        OF.bump_weight_generation()
        self.calls += 1
        return loss[0]

    def phase_us(self):
        """Phase durations of the last step from :attr:`stamps` (synchronises; re-zeroes the latest-workgroup half):
        [(name, workgroup 0 us, latest workgroup us), ...] -- the latest workgroup's column is the time from the
        previous boundary's latest arrival to this one's."""
        t = self.stamps.tolist()
        self.stamps[64:].zero_()
        nl = len(self.layers)
        names = []
        for l in range(nl - 1):
            names += [f"F{l}", f"bar F{l}"]
        names += ["CE", "bar CE"]
        fused = self.fused_update()
        for j in range(nl - 1, 0, -1):
            if fused:
                win = f"B{j} arrive+wgrad+update L{j}" + (f" (+W^T L{j + 1})" if j + 1 < nl else "")
            else:
                win = f"B{j} arrive+wgrad+update L{j + 1}" if j + 1 < nl else f"B{j} arrive+wgrad"
            names += [f"B{j} dgrad", win, f"bar B{j} wait"]
        names += ["B0 wgrad+update L0 (+W^T L1)", "-"] if fused else ["B0 wgrad", "update L1 + L0"]
        out = []
        for i, n in enumerate(names):
            out.append((n, (t[i + 1] - t[i]) / 100.0, (t[64 + i + 1] - t[64 + i]) / 100.0 if i > 0 else 0.0))
        return out

    def fused_update(self) -> bool:
        """Whether the kernel updates each weight tile straight from its gradient accumulators, in the same window
        (Adam / AdamW and every layer's 64x64 gradient tiles within the grid; ``PDE_MLP_FUSE=0`` turns it off) --
        else one window later, reading the gradient back (the form SGD keeps)."""
        if self.mode == 0 or os.environ.get("PDE_MLP_FUSE", "1") == "0":
            return False
        g = self.grid()
        return all(-(-L.out_features // 64) * -(-L.in_features // 64) <= g for L in self.layers)

    def check(self, where: str = "") -> None:
        """Raise :class:`DeviceBarrierError` if a grid barrier timed out since the last check (synchronises), and
        RuntimeError if an in-launch exchange timed out waiting for a peer."""
        if self.xgmi is not None:
            self.xgmi.check()
        n = self.errors()
        if n:
            raise DeviceBarrierError(f"MegaMLP: {n} grid-barrier timeout(s){' at ' + where if where else ''}: a "
                                     "workgroup was not resident, the step's hand-offs raced")

    def errors(self) -> int:
        """Non-zero if a grid barrier of a step timed out (a workgroup could not be resident): synchronises.  The
        barrier counters run across launches; after a timeout they are re-zeroed here (with the error word)."""
        n = 0
        for b in self._bufs.values():
            e = int(b["err"].item())
            if e:
                b["bar"].zero_()
                b["err"].zero_()
            n += e
        return n

    @staticmethod
    def kernel_launches_per_step() -> int:
        return 1
