"""Autograd functions over the gfx950 HIP kernels (``_C``), with a plain-PyTorch CPU path.

Device policy
-------------
* GPU tensors take the native path: activations are bf16, convolutions are NHWC (channels padded to a
  multiple of 8 with zeros), every matmul-shaped op runs on the MFMA implicit-GEMM kernel and the
  element-wise/normalisation work on the fused kernels of ``csrc/kernels``.  The extension is required;
  a missing build raises (``_native.NativeUnavailable``) instead of silently using ATen.
* CPU tensors take the reference path (fp32 NCHW ``torch.nn.functional``), which is what the
  reference scripts run (every reference workload is CPU/gloo) and what the CPU/gloo
  config of BASELINE.json (config 0) measures.

Parameters always stay in PyTorch's fp32 layout (``Linear.weight`` [out, in], ``Conv2d.weight``
[Co, Ci, R, S]) so ``state_dict``s interoperate with the reference's snapshot format
(pytorch_elastic/mnist_ddp_elastic.py:95-104).  The bf16 / re-laid-out compute copies are produced by
small layout kernels and cached per (parameter version, optimiser generation).
"""
from __future__ import annotations

import contextlib
import math
import threading

import torch
import torch.nn.functional as F

from .. import _native
from . import streams

# ---------------------------------------------------------------------------------------------
# compute-copy cache
# ---------------------------------------------------------------------------------------------
_GEN = [0]
_FORCE_RECOMPUTE = [False]


def bump_weight_generation() -> None:
    """Invalidate all cached bf16 compute copies (called by the fused optimiser after a step)."""
    _GEN[0] += 1


def weight_generation() -> int:
    """Current weight generation (changes whenever an optimiser step may have written the weights)."""
    return _GEN[0]


class recompute_weight_copies:
    """Context manager: never reuse cached copies (used while capturing a hipGraph so the layout
    kernels become part of the graph and see every replay's updated weights)."""

    def __enter__(self):
        self._old = _FORCE_RECOMPUTE[0]
        _FORCE_RECOMPUTE[0] = True

    def __exit__(self, *exc):
        _FORCE_RECOMPUTE[0] = self._old


def _cached(p: torch.Tensor, kind, fn):
    if _FORCE_RECOMPUTE[0]:
        return fn()
    key = (p._version, _GEN[0])
    cache = p.__dict__.setdefault("_pde_cache", {})
    ent = cache.get(kind)
    if ent is None or ent[0] != key:
        ent = (key, fn())
        cache[kind] = ent
    return ent[1]


_EMU = [False]


class emulate_bf16_on_cpu:
    """Context manager for numerics tests: the CPU reference path rounds weights, inputs and outputs of
    every op to bf16 like the GPU kernels store them (fp32 math in between), so GPU-vs-CPU differences
    isolate kernel bugs from bf16 storage noise."""

    def __enter__(self):
        self._old = _EMU[0]
        _EMU[0] = True

    def __exit__(self, *exc):
        _EMU[0] = self._old


def _emu(t):
    if t is None or not _EMU[0]:
        return t
    return t.to(torch.bfloat16).to(t.dtype)


def pad8(c: int) -> int:
    return (c + 7) // 8 * 8


def _C():
    return _native.C()


class DeviceHandoffError(RuntimeError):
    """A one-launch BatchNorm's cross-block hand-off timed out on the device (norm_pool.hip error word):
    the normalisation of that step used incomplete statistics, so the replica's state is not trustworthy."""


def check_device_errors(where: str = "") -> None:
    """Read (and reset) the one-launch BatchNorm error word at a sync point; raise :class:`DeviceHandoffError`
    if any flag / tagged-partial wait timed out since the last check.  Synchronises the device (call it only
    where the host already waits: end of a timed region, epoch end, pipeline ``check()``).  No-op without a
    GPU or before the native library was loaded."""
    if not torch.cuda.is_available() or not _native.loaded("_C"):
        return
    v = _native.C().bn_error(True)
    if v != 0:
        raise DeviceHandoffError(f"one-launch BatchNorm hand-off {'failed' if v < 0 else 'timed out'} "
                                 f"(error word {v}){' at ' + where if where else ''}: statistics of the step are "
                                 "incomplete; the grid was not co-resident (PDE_BN_FUSED=0 disables the one-launch path)")


# ---------------------------------------------------------------------------------------------
# GEMM pairing
# ---------------------------------------------------------------------------------------------
class BnHeadroom:
    """CUs reserved, for this object's lifetime, for kernels that keep spinning on OTHER streams of this process
    while a one-launch BatchNorm may run -- a pipeline channel's ring sends waiting for credit, an overlapped RCCL
    all-reduce (csrc/kernels/norm_pool.hip bn_reserve_headroom): the BatchNorm's grid shrinks to the remaining
    resident cap, and a BatchNorm whose smallest grid does not fit is refused up front (multi-launch) instead of
    timing out in its flag waits.  GPU only (a no-op without the native extension)."""

    def __init__(self, blocks: int):
        self.blocks = max(0, int(blocks))
        self.cap = None
        if self.blocks and torch.cuda.is_available():
            self.cap = _C().bn_reserve_headroom(self.blocks)
        else:
            self.blocks = 0

    def release(self):
        if self.blocks:
            _C().bn_reserve_headroom(-self.blocks)
            self.blocks = 0

    def __del__(self):
        try:
            self.release()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def bn_launch_stats() -> dict:
    """One-launch / multi-launch BatchNorm counts, the last one-launch grid and the current resident cap."""
    return dict(_C().bn_launch_stats())


class gemm_pair:
    """Context manager: the (at most two) GEMM ops issued inside are launched together as ONE paired launch
    when the block exits (``pde::gemm_bf16_pair``: the first op's tiles are scheduled first; both grids fill
    the chip together and pay one launch boundary).  Ops inside must not read each other's outputs; non-GEMM
    kernels issued inside run immediately (before the pair).  ``PDE_GEMM_PAIR=0`` launches them one by one.
    ``defer_second=True``: the second op is a weight gradient accumulated into ``.grad``; its split-K slab
    reduction joins the step's single batched reduction (:func:`.streams.flush_deferred`)."""

    def __init__(self, defer_second: bool = False, flush_by_caller: bool = False):
        self.defer = defer_second and streams.defer_enabled()
        self.flush_by_caller = flush_by_caller

    def __enter__(self):
        _C().gemm_pair_begin()
        return self

    def __exit__(self, exc_type, *exc):
        if _C().gemm_pair_end(exc_type is not None, self.defer):
            streams.note_deferred_reduce(self.flush_by_caller)


# ---------------------------------------------------------------------------------------------
# direct gradient accumulation
# ---------------------------------------------------------------------------------------------
_DIRECT_GRAD = [True]


class direct_grad_accumulation:
    """Context manager toggling direct accumulation (default on): weight-gradient kernels add into an
    existing ``param.grad`` themselves instead of returning a fresh tensor that autograd then adds --
    one gradient tensor and one add kernel less per parameter and step.  The backward then returns
    ``None`` for that parameter; autograd still runs the parameter's AccumulateGrad node, so
    post-accumulate-grad hooks (DDP / Horovod overlap) fire exactly as before, after the kernel that
    accumulated the gradient has been enqueued (tests/test_kernels_gpu.py::test_direct_grad_accumulation)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled

    def __enter__(self):
        self._old = _DIRECT_GRAD[0]
        _DIRECT_GRAD[0] = self.enabled

    def __exit__(self, *exc):
        _DIRECT_GRAD[0] = self._old


def _sink_accum(g) -> bool:
    """Whether a kernel writing into the gradient sink ``g`` must ADD: False for the first writer after a
    zero-filling ``zero_grad`` (parallel/ddp.py marks the views) -- it stores, bitwise the same as adding to zero,
    without reading the gradient back (the scattered OIHW epilogues read-modify-wrote every element)."""
    return not g.__dict__.pop("_pde_fresh", False)


def _grad_sink(p):
    """``p.grad`` when a kernel may accumulate straight into it, else None (return the grad to autograd)."""
    if p is None or not _DIRECT_GRAD[0]:
        return None
    g = p.grad
    if (g is None or g.dtype != torch.float32 or g.device != p.device or g.shape != p.shape
            or not g.is_contiguous() or g.requires_grad):
        return None
    return g


# ---------------------------------------------------------------------------------------------
# optimizer-maintained compute copies
# ---------------------------------------------------------------------------------------------
def maintain_compute_copies(p: torch.Tensor):
    """Allocate the bf16 compute copies of a GPU weight that the fused optimizer keeps in sync from now on.
    Covered: linear weights (``_pde_linear``) and 1x1 conv weights (``_pde_conv``) with channel counts that
    need no padding -- for those the implicit-GEMM forward layout [Co, Ci] IS the OIHW order, the optimizer
    writes the copy in the same launch as the update (contiguous stores) and the dgrad GEMM reads it
    transposed; and every other conv weight (3x3, 7x7, padded channels): its forward [Cop, R*S*Cp] and
    dgrad [Cp, R*S*Cop] layouts (key ``"kxk"`` = (Cp, Cop)), refreshed for all such weights by ONE
    multi-tensor launch after the update (``conv_layouts_step``) instead of two conversion kernels per
    conv and step.  Returns the copy dict (or None).  The copies are tied to the weight's version counter:
    an in-place write outside the optimizer (load_state_dict, a broadcast, an elastic restore) is detected
    by :func:`_maintained` and the copies are re-derived in place.  A parameter marked ``_pde_own_copies`` (its
    consumer keeps its own operand image, e.g. the fused CNN's bf16 fragment image rebuilt in-kernel) gets none:
    the optimiser then skips their refresh (the 14 us conv-layout launch of the Horovod-elastic AdamW step)."""
    if not p.is_cuda or p.dtype != torch.float32 or p.__dict__.get("_pde_own_copies", False):
        return None
    d = {}
    if getattr(p, "_pde_conv", False) and p.dim() == 4:
        co, ci, r, s = p.shape
        if r * s == 1 and ci % 8 == 0 and co % 8 == 0:
            d["bf16"] = torch.empty(p.shape, dtype=torch.bfloat16, device=p.device)
            d["conv_fwd"] = d["bf16"].view(co, ci)
        else:
            cp, cop = pad8(ci), pad8(co)
            d["kxk"] = (cp, cop)
            d["conv_fwd"] = torch.empty(cop, r * s * cp, dtype=torch.bfloat16, device=p.device)
            d["conv_dgrad"] = torch.empty(cp, r * s * cop, dtype=torch.bfloat16, device=p.device)
    elif getattr(p, "_pde_linear", False) and p.dim() == 2:
        out_f = p.shape[0]
        if out_f % 8 == 0:
            d["bf16"] = torch.empty(p.shape, dtype=torch.bfloat16, device=p.device)
        else:
            # rows padded to a multiple of 8 with zeros (written once, never by the optimizer): the dgrad GEMM
            # can take the padded copy as a K = pad8(out) operand on the FAST path (models/mlp_fused.py)
            pad = torch.zeros(pad8(out_f), p.shape[1], dtype=torch.bfloat16, device=p.device)
            d["bf16_pad"] = pad
            d["bf16"] = pad[:out_f]
    else:
        return None
    _derive_copies(p, d)
    d["version"] = p._version
    p.__dict__["_pde_maint"] = d
    return d


def _derive_copies(p: torch.Tensor, d: dict):
    w = p.detach().contiguous()
    if "kxk" in d:
        cp, cop = d["kxk"]
        _C().conv_w_fwd(w, cp, cop, d["conv_fwd"])
        _C().conv_w_dgrad(w, cp, cop, d["conv_dgrad"])
    else:
        _C().cast_bf16_into(w, d["bf16"])
    if "bf16_t" in d:  # the transposed copy (models/mlp_mega.py: the dgrad operand), padded columns stay zero
        d["bf16_t"][:, :w.shape[0]].copy_(w.t())


def maintain_transposed_copy(p: torch.Tensor, ldt: int) -> torch.Tensor:
    """Also keep a transposed bf16 copy [in, ldt] (columns past ``out`` zero) of a linear weight in sync: the fused
    MLP step (mlp_fused.hip) refreshes it with the update and reads it as the data-gradient operand; a write
    outside it is detected by the version counter like the other copies (:func:`_maintained`)."""
    d = p.__dict__.get("_pde_maint") or maintain_compute_copies(p)
    if d is None:
        raise ValueError("maintain_transposed_copy: a GPU fp32 linear weight is required")
    t = d.get("bf16_t")
    if t is None or t.shape[1] != ldt:
        d["bf16_t"] = torch.zeros(p.shape[1], ldt, dtype=torch.bfloat16, device=p.device)
        _derive_copies(p, d)
        d["version"] = p._version
    return _maintained(p, "bf16_t")


def release_compute_copies(p: torch.Tensor) -> None:
    """Stop treating ``p``'s bf16 compute copies as optimizer-maintained: an update path that writes the
    fp32 weights without refreshing them (the fused CNN step keeps its own fragment image) must not leave
    the layers reading stale copies; the layers fall back to generation-keyed cached copies."""
    p.__dict__.pop("_pde_maint", None)


def _maintained(p: torch.Tensor, kind: str):
    """The optimizer-maintained copy ``kind`` of ``p`` (None if the optimizer does not maintain one)."""
    d = p.__dict__.get("_pde_maint")
    if d is None or kind not in d:
        return None
    if d["version"] != p._version:  # written outside the optimizer: re-derive in place
        _derive_copies(p, d)
        d["version"] = p._version
    return d[kind]


def _bf16_weight(w: torch.Tensor) -> torch.Tensor:
    m = _maintained(w, "bf16")
    if m is not None:
        return m
    return _cached(w, "bf16", lambda: _C().cast_bf16(w.detach().contiguous()))


# ---------------------------------------------------------------------------------------------
# Linear (+ bias, + ReLU): y = relu?(x W^T + b)
# ---------------------------------------------------------------------------------------------
class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu, out_f32, consumer_masks, mask_input_grad):
        wb = _bf16_weight(weight)
        y = _C().linear_fwd(x, wb, bias.detach() if bias is not None else None, relu, out_f32)
        ctx.relu = relu and not consumer_masks
        ctx.mask_input_grad = mask_input_grad
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)
        ctx.save_for_backward(x, wb, y if ctx.relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb, y = ctx.saved_tensors
        dy = dy.contiguous()
        if dy.dtype != torch.bfloat16:
            dy = _C().cast_bf16(dy.float().contiguous())
        if ctx.relu:
            dy = _C().relu_bwd(dy, y)
        dx = dw = db = None
        weight, bias = ctx.params
        wsink = _grad_sink(weight) if ctx.needs_input_grad[1] else None
        bsink = _grad_sink(bias) if ctx.has_bias and ctx.needs_input_grad[2] else None
        if wsink is not None and ctx.needs_input_grad[0] and not streams.active_for(dy):
            # dgrad + wgrad as ONE paired GEMM launch (the dgrad's tiles first: it feeds the next layer)
            with gemm_pair(defer_second=True):
                dx = _C().linear_dgrad(dy, wb, x if ctx.mask_input_grad else None)
                _C().linear_wgrad(dy, x, wsink, _sink_accum(wsink))
            if bsink is not None:
                _C().colsum(dy, -1, bsink, _sink_accum(bsink))
            elif ctx.has_bias and ctx.needs_input_grad[2]:
                db = _C().colsum(dy, -1, None, False)
            return dx, None, db, None, None, None, None
        if wsink is not None and (bsink is not None or not ctx.has_bias or not ctx.needs_input_grad[2]) \
                and ctx.needs_input_grad[0] and streams.active_for(dy):
            # weight / bias gradients go straight into .grad on the side stream, concurrent with the dgrad
            with streams.fork(dy, x):
                _C().linear_wgrad(dy, x, wsink, _sink_accum(wsink))
                if bsink is not None:
                    _C().colsum(dy, -1, bsink, _sink_accum(bsink))
            dx = _C().linear_dgrad(dy, wb, x if ctx.mask_input_grad else None)
            return dx, None, None, None, None, None, None
        if ctx.needs_input_grad[0]:
            dx = _C().linear_dgrad(dy, wb, x if ctx.mask_input_grad else None)
        if ctx.needs_input_grad[1]:
            dw = _C().linear_wgrad(dy, x, wsink, wsink is not None and _sink_accum(wsink))
            if wsink is not None:
                dw = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _C().colsum(dy, -1, bsink, bsink is not None and _sink_accum(bsink))
            if bsink is not None:
                db = None
        return dx, dw, db, None, None, None, None


def linear(x, weight, bias=None, relu=False, out_f32=False, consumer_masks=False, mask_input_grad=False):
    """Fused linear layer.

    GPU: bf16 MFMA GEMM with bias/ReLU fused in the epilogue.  ``consumer_masks`` declares that the
    next layer's backward already applies this layer's ReLU mask (its ``mask_input_grad``), which
    fuses threshold_backward into the dgrad GEMM epilogue (SURVEY.md §2.5 MLP table).
    """
    if not x.is_cuda:
        y = F.linear(_emu(x), _emu(weight), bias)
        y = F.relu(y) if relu else y
        return y if out_f32 else _emu(y)
    if x.dtype != torch.bfloat16:
        x = _C().cast_bf16(x.float().contiguous())
    return _LinearFn.apply(x.contiguous(), weight, bias, relu, out_f32, consumer_masks, mask_input_grad)


# ---------------------------------------------------------------------------------------------
# NHWC implicit-GEMM convolution
# ---------------------------------------------------------------------------------------------
def _conv_fwd_weight(x, weight):
    """The forward implicit-GEMM copy of a conv weight ([Cop, R*S*Cp] bf16) for input ``x``."""
    co, ci, r, s = weight.shape
    cp = x.shape[3]
    cop = pad8(co)
    wf = _maintained(weight, "conv_fwd") if cp == pad8(ci) else None
    if wf is None:
        wf = _cached(weight, ("conv_fwd", cp, cop), lambda: _C().conv_w_fwd(weight.detach().contiguous(), cp, cop))
    return wf


class _ConvBwdCtx:
    """What :func:`_conv_backward` needs of a conv's autograd context (shared by the plain conv and the
    conv with a BatchNorm folded into its input)."""
    __slots__ = ("join", "grad_to", "geom", "relu", "has_bias", "bias", "needs_input_grad")


class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, relu, join=None, grad_to=None, defer=False, stats=None,
                dx_defer=False):
        ctx.join = join
        ctx.grad_to = grad_to
        ctx.dx_defer = dx_defer
        co, ci, r, s = weight.shape
        cp = x.shape[3]
        cop = pad8(co)
        wf = _conv_fwd_weight(x, weight)
        if stats is not None:
            # producer of a folded BatchNorm: the epilogue emits the output's statistics and the launch's last
            # block finalizes that BatchNorm (mean / invstd / scale-shift / running statistics) into `stats`
            y = stats.produce(x, wf, r, s, stride, pad)
        else:
            # defer: a split-K GEMM leaves its slabs for the BatchNorm that follows (it reduces them itself)
            y = _C().conv_fwd(x, wf, bias.detach() if bias is not None else None, r, s, stride, pad, relu, False,
                              defer)
        ctx.geom = (co, ci, r, s, stride, pad, cp, cop, x.shape[1], x.shape[2])
        ctx.relu = relu
        ctx.has_bias = bias is not None
        ctx.bias = bias
        ctx.save_for_backward(x, weight, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        dx, dw, db = _conv_backward(ctx, dy, x, weight, y)
        return dx, dw, db, None, None, None, None, None, None, None, None


def _conv_backward(ctx, dy, x, weight, y=None):
    """dx, dw, db of a conv (dgrad + wgrad as one paired launch, or wgrad on the side stream); ``ctx`` carries
    join / grad_to / geom / relu / has_bias / bias / needs_input_grad (x, weight, bias)."""
    if True:
        co, ci, r, s, stride, pad, cp, cop, h, w = ctx.geom
        dy = dy.contiguous()
        if ctx.relu:
            dy = _C().relu_bwd(dy, y)
        dx = dw = db = None
        wsink = _grad_sink(weight) if ctx.needs_input_grad[1] else None
        bsink = _grad_sink(ctx.bias) if ctx.has_bias and ctx.needs_input_grad[2] else None
        side = (wsink is not None and ctx.needs_input_grad[0] and streams.active_for(dy)
                and (bsink is not None or not ctx.has_bias or not ctx.needs_input_grad[2]))
        if side:
            # the weight (and bias) gradient is off the critical path: side stream, issued BEFORE the dgrad so
            # the fork point does not wait for it (ops/streams.py)
            with streams.fork(dy, x):
                _C().conv_wgrad(dy, x, r, s, stride, pad, co, ci, wsink, _sink_accum(wsink))
                if bsink is not None:
                    _C().colsum(dy, co, bsink, _sink_accum(bsink))
        paired = wsink is not None and ctx.needs_input_grad[0] and not side
        if paired:
            # dgrad + wgrad as ONE paired GEMM launch (dgrad tiles first); the dgrad op is issued first
            pair = gemm_pair(defer_second=True)
            pair.__enter__()
        if ctx.needs_input_grad[0]:
            # residual fork: the other branch's gradient (stored by the block's last BatchNorm) is added in the
            # dgrad epilogue instead of by a separate autograd add
            other = ctx.join.take() if ctx.join is not None else None
            # dx_defer (the conv's input is a BatchNorm + ReLU output consumed by this conv alone): a split-K
            # dgrad leaves its slabs for that BatchNorm's backward, which sums them itself (no reduce launch)
            defer = (paired and other is None and ctx.grad_to is None and getattr(ctx, "dx_defer", False)
                     and _BN_BWD_DEFER[0])
            wf = _maintained(weight, "conv_fwd") if (r == 1 and s == 1 and pad == 0) else None
            if wf is not None and weight.__dict__["_pde_maint"].get("kxk") is None:
                # 1x1 (stride 1 or 2): the dgrad GEMM reads the forward copy [Co, Ci] transposed
                dx = _C().conv_dgrad(dy, wf, h, w, r, s, stride, pad, other, True, other is not None, defer)
            else:
                wd = _maintained(weight, "conv_dgrad") if cp == pad8(ci) else None
                if wd is None:
                    wd = _cached(weight, ("conv_dgrad", cp, cop),
                                 lambda: _C().conv_w_dgrad(weight.detach().contiguous(), cp, cop))
                dx = _C().conv_dgrad(dy, wd, h, w, r, s, stride, pad, other, False, other is not None, defer)
            if ctx.grad_to is not None:  # the other consumer of x adds this gradient in its dgrad epilogue
                ctx.grad_to.put(dx)
                dx = None
        if paired:
            try:
                _C().conv_wgrad(dy, x, r, s, stride, pad, co, ci, wsink, _sink_accum(wsink))
            except BaseException as exc:
                pair.__exit__(type(exc), exc, None)
                raise
            pair.__exit__(None, None, None)
            if ctx.has_bias and ctx.needs_input_grad[2]:
                db = _C().colsum(dy, co, bsink, bsink is not None and _sink_accum(bsink))
                if bsink is not None:
                    db = None
            return dx, None, db
        if side:
            return dx, None, None
        if ctx.needs_input_grad[1]:
            # OIHW epilogue: the GEMM writes the parameter's layout (and adds into .grad when it exists)
            dw = _C().conv_wgrad(dy, x, r, s, stride, pad, co, ci, wsink, wsink is not None and _sink_accum(wsink))
            if wsink is not None:
                dw = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _C().colsum(dy, co, bsink, bsink is not None and _sink_accum(bsink))
            if bsink is not None:
                db = None
        return dx, dw, db


class GradJoin:
    """Hand-off of one gradient between the two consumers of a residual fork (GPU training).

    In a bottleneck block without downsample, the block input feeds conv1 and the residual of the last
    BatchNorm.  Passing the same ``GradJoin`` to ``batch_norm(..., residual_grad_to=j)`` and
    ``conv2d(..., grad_join=j)`` makes the BatchNorm backward hand its residual gradient to the join
    (instead of returning it to autograd), and conv1's dgrad GEMM adds it in its epilogue: one bf16 add kernel
    and one gradient tensor fewer per block.  Autograd order is guaranteed by data dependence: conv1's
    backward needs the gradient that flows back through the BatchNorm.

    In a block WITH downsample, the block input feeds conv1 and the downsample conv:
    ``conv2d(x, ..., grad_to=j)`` on the downsample conv hands ITS data gradient to the join and conv1's
    dgrad adds it -- the bf16 add autograd would run for the two gradients of x.  Order: the downsample
    branch's nodes are created after conv2/bn2 in forward, so the engine (higher sequence number first among
    ready nodes) runs the downsample conv's backward before bn2 -> conv2 -> bn1 -> conv1's; ``take`` asserts
    it."""

    __slots__ = ("grad",)

    def __init__(self):
        self.grad = None

    def put(self, g):
        self.grad = g

    def take(self):
        g, self.grad = self.grad, None
        return g


def conv2d(x, weight, bias=None, stride=1, padding=0, relu=False, grad_join=None, grad_to=None, bn_follows=False,
           bn_stats=None, dx_bn=False):
    """2-D convolution.  GPU: ``x`` is NHWC bf16 with C padded to a multiple of 8; output NHWC with
    Cout padded to a multiple of 8 (padded channels are exactly zero).  CPU: NCHW fp32 F.conv2d.
    ``grad_join`` (this conv's dgrad adds the join's gradient) / ``grad_to`` (this conv's input gradient
    goes to the join instead of autograd): see :class:`GradJoin` (GPU only; ignored on CPU).
    ``bn_follows``: a training-mode batch_norm consumes the output next -- a split-K GEMM then skips its
    slab reduction and the one-launch BatchNorm sums the slabs itself (any other reader resolves them).
    ``dx_bn``: ``x`` is a training BatchNorm(+ReLU) output that ONLY this conv consumes -- the backward's split-K
    dgrad then leaves its slabs for that BatchNorm's backward in the same way (the caller vouches for the
    single consumer: an autograd accumulation of the pending gradient would read it unreduced)."""
    if not x.is_cuda:
        y = F.conv2d(_emu(x), _emu(weight), bias, stride=stride, padding=padding)
        return _emu(F.relu(y) if relu else y)
    defer = bool(bn_follows) and bias is None and not relu and _DEFER_CONV[0]
    return _Conv2dFn.apply(x.contiguous(), weight, bias, int(stride), int(padding), relu, grad_join, grad_to, defer,
                           bn_stats, bool(dx_bn))


import os as _os

_DEFER_CONV = [_os.environ.get("PDE_CONV_BN_DEFER", "1") != "0"]  # A/B switch
_BN_BWD_DEFER = [_os.environ.get("PDE_BN_BWD_DEFER", "1") != "0"]  # A/B switch: dgrad slabs summed by bn_bwd


def to_native_image(x: torch.Tensor) -> torch.Tensor:
    """NCHW fp32 input batch -> the device's native activation layout (NHWC bf16 padded on GPU)."""
    if not x.is_cuda:
        return _emu(x)
    return _C().nchw_to_nhwc(x.float().contiguous(), pad8(x.shape[1]))


# ---------------------------------------------------------------------------------------------
# BatchNorm2d (train: batch statistics; eval: running statistics), fused residual add + ReLU
# ---------------------------------------------------------------------------------------------
_BN_GROUPS = threading.local()


@contextlib.contextmanager
def bn_groups(groups: int):
    """Training-mode BatchNorm inside this context normalises ``groups`` equal, contiguous slices of the
    batch (micro-batches) with their OWN statistics, in one launch per layer; running statistics get the
    ``groups`` momentum updates in slice order.  A pipeline stage runs several micro-batches per launch this
    way and keeps the per-micro-batch BatchNorm semantics of the reference (``split_size``, quirk Q17):
    identical results to ``groups`` separate forward passes, at the launch count of one."""
    prev = getattr(_BN_GROUPS, "g", 1)
    _BN_GROUPS.g = int(groups)
    try:
        yield
    finally:
        _BN_GROUPS.g = prev


def current_bn_groups() -> int:
    return getattr(_BN_GROUPS, "g", 1)


class _BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, residual, eps, momentum, relu, join=None,
                groups=1):
        ctx.join = join
        ctx.groups = groups
        y, mean, invstd, ss = _C().bn_fwd(x, gamma.detach() if gamma is not None else None,
                                          beta.detach() if beta is not None else None, running_mean,
                                          running_var, eps, momentum, residual, relu, groups)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.beta = beta
        # without a residual the backward recomputes the ReLU mask from x with the forward's scale/shift
        ctx.save_for_backward(x, y, mean, invstd, gamma, ss)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, invstd, gamma, ss = ctx.saved_tensors
        beta = ctx.beta
        dg_sink, db_sink = _grad_sink(gamma), _grad_sink(beta)
        direct = dg_sink is not None and db_sink is not None
        # both sinks are first written here or both were written before (pop both marks: no short-circuit)
        accum = (_sink_accum(dg_sink) | _sink_accum(db_sink)) if direct else True
        dx, dg, db, dres = _C().bn_bwd(dy.contiguous(), x, y, mean, invstd,
                                       gamma.detach() if gamma is not None else None, ctx.relu, ctx.has_res,
                                       dg_sink if direct else None, db_sink if direct else None,
                                       None if ctx.has_res else ss, ctx.groups, accum)
        if direct:  # dgamma / dbeta were added into .grad by the finalize kernel
            dg = db = None
        if ctx.has_res and ctx.join is not None:  # the residual fork's conv adds it in its dgrad epilogue
            ctx.join.put(dres)
            dres = None
        return dx, dg, db, None, None, (dres if ctx.has_res else None), None, None, None, None, None


def batch_norm(x, weight, bias, running_mean, running_var, training, momentum=0.1, eps=1e-5, residual=None,
               relu=False, residual_grad_to=None):
    """BatchNorm2d with optional fused residual add and ReLU:  relu?(bn(x) + residual).
    ``residual_grad_to``: a :class:`GradJoin` that receives the residual's gradient (GPU training only)."""
    groups = current_bn_groups() if training else 1
    if not x.is_cuda:
        if groups > 1:  # per-slice statistics, running stats updated slice by slice (in order)
            y = torch.cat([F.batch_norm(xs, running_mean, running_var, weight, bias, True, momentum, eps)
                           for xs in x.chunk(groups)])
        else:
            y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
        if residual is not None:
            y = y + residual
        return _emu(F.relu(y) if relu else y)
    x = x.contiguous()
    if training:
        return _BatchNormFn.apply(x, weight, bias, running_mean, running_var,
                                  residual.contiguous() if residual is not None else None, eps, momentum, relu,
                                  residual_grad_to if residual is not None else None, groups)
    invstd = torch.rsqrt(running_var + eps)
    scale = (weight * invstd if weight is not None else invstd).float().contiguous()
    shift = ((bias if bias is not None else 0) - running_mean * scale).float().contiguous()
    return _C().bn_apply(x, scale, shift, residual.contiguous() if residual is not None else None, relu)


# ---------------------------------------------------------------------------------------------
# BatchNorm folded into the convolutions around it (training, GPU; csrc/kernels/gemm.hip BnFoldIn / BnStatsOut)
# ---------------------------------------------------------------------------------------------
# Opt-in (PDE_BN_FOLD=1). Measured on MI355X (profiles/r4h_bnfold_ab_bench.jsonl, README "BatchNorm fold"):
# ResNet-50 bs32 step 3.55 ms folded vs 3.29 ms unfolded -- the producer's last-block finalize tail (~7.5 us)
# and the consumer's A transform (~3.8 us) cost more than the BatchNorm launches they remove (~0.03 ms total).
_BN_FOLD = [_os.environ.get("PDE_BN_FOLD", "0") == "1"]


def bn_fold_enabled() -> bool:
    return _BN_FOLD[0]


def bn_fold_buffers(bn, groups: int):
    """The persistent (self-cleaning) statistics buffer [shards, G, 2, C] int64 + arrival ticket of BatchNorm
    ``bn``: the producer conv's epilogue adds into it, the producer launch's last block reads-and-zeroes it."""
    bufs = bn.__dict__.setdefault("_pde_fold", {})
    if groups not in bufs:
        dev = bn.weight.device
        shards = _C().bn_fold_shards()  # row-tile shards of the sums (contention, see pde_kernels.h)
        bufs[groups] = (torch.zeros(shards * groups * 2 * bn.num_features, dtype=torch.long, device=dev),
                        torch.zeros(1, dtype=torch.int32, device=dev))
    return bufs[groups]


class BnFoldStats:
    """One training-mode BatchNorm2d ``bn`` folded into the convs around it, for one forward: the producer conv
    (``conv2d(..., bn_stats=this)``) emits and finalizes its statistics -- :meth:`produce` keeps the saved mean /
    invstd / scale-shift -- and :func:`bn_relu_conv` applies it in the consumer conv's A loader."""

    def __init__(self, bn, groups: int):
        self.bn, self.groups = bn, groups
        self.sums, self.ticket = bn_fold_buffers(bn, groups)
        self.mean = self.invstd = self.ss = None

    def produce(self, x, wf, r, s, stride, pad):
        bn = self.bn
        y, self.mean, self.invstd, self.ss, _ = _C().conv_fwd_bn(
            x, wf, r, s, stride, pad, self.groups, self.sums, self.ticket, bn.weight.detach(), bn.bias.detach(),
            bn.running_mean, bn.running_var, bn.eps, bn.momentum, None, False, False)
        bn._nbt_pending += self.groups
        return y


class _BnConvFn(torch.autograd.Function):
    """conv(relu(bn(a))) with the BatchNorm (+ ReLU) applied in the conv's A loader from the scale / shift the
    producer of ``a`` finalized; the activation is written once by the conv (the backward's operand).
    Backward: the conv's dgrad / wgrad against that activation, then the BatchNorm backward (ReLU mask from
    ``a`` and the saved scale / shift)."""

    @staticmethod
    def forward(ctx, a, gamma, beta, weight, st, relu, stride, pad, stats_out=None, defer=False):
        co, ci, r, s = weight.shape
        cp = a.shape[3]
        wf = _conv_fwd_weight(a, weight)
        if stats_out is not None:  # this conv also produces the NEXT BatchNorm's statistics
            y = stats_out.produce_folded(a, wf, r, s, stride, pad, st.ss, relu)
            act = stats_out.act
        else:
            y, _, _, _, act = _C().conv_fwd_bn(a, wf, r, s, stride, pad, st.groups, None, None, None, None, None,
                                               None, 0.0, 0.0, st.ss, relu, defer)
        ctx.geom = (co, ci, r, s, stride, pad, cp, pad8(co), a.shape[1], a.shape[2])
        ctx.relu, ctx.groups = relu, st.groups
        ctx.beta = beta
        ctx.save_for_backward(a, act, st.mean, st.invstd, gamma, st.ss, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        a, act, mean, invstd, gamma, ss, weight = ctx.saved_tensors
        cx = _ConvBwdCtx()
        cx.join = cx.grad_to = None
        cx.geom, cx.relu, cx.has_bias, cx.bias = ctx.geom, False, False, None
        cx.needs_input_grad = (True, ctx.needs_input_grad[3], False)
        dact, dw, _ = _conv_backward(cx, dy, act, weight)
        beta = ctx.beta
        dg_sink, db_sink = _grad_sink(gamma), _grad_sink(beta)
        direct = dg_sink is not None and db_sink is not None
        accum = (_sink_accum(dg_sink) | _sink_accum(db_sink)) if direct else True
        da, dg, db, _ = _C().bn_bwd(dact, a, act, mean, invstd, gamma.detach(), ctx.relu, False,
                                    dg_sink if direct else None, db_sink if direct else None, ss, ctx.groups,
                                    accum)
        if direct:
            dg = db = None
        return da, dg, db, dw, None, None, None, None, None, None


def _produce_folded(self, a, wf, r, s, stride, pad, fold_ss, relu):
    """BnFoldStats.produce for a conv that itself consumes a folded BatchNorm (both sides in one launch)."""
    bn = self.bn
    y, self.mean, self.invstd, self.ss, self.act = _C().conv_fwd_bn(
        a, wf, r, s, stride, pad, self.groups, self.sums, self.ticket, bn.weight.detach(), bn.bias.detach(),
        bn.running_mean, bn.running_var, bn.eps, bn.momentum, fold_ss, relu, False)
    bn._nbt_pending += self.groups
    return y


BnFoldStats.produce_folded = _produce_folded


def bn_relu_conv(a, st: BnFoldStats, conv, relu=True, stats_out: BnFoldStats | None = None, bn_follows=False):
    """``conv(relu(st.bn(a)))`` for the BatchNorm whose statistics the producer of ``a`` emitted
    (``conv2d(..., bn_stats=st)``) and a bias-free Conv2d ``conv`` (a 1x1, or a 3x3 of stride 1).
    ``stats_out``: this conv's epilogue also emits (and finalizes) the NEXT BatchNorm."""
    assert st.ss is not None, "the producer conv of this BatchNorm has not run"
    bn = st.bn
    defer = bool(bn_follows) and stats_out is None and _DEFER_CONV[0]
    return _BnConvFn.apply(a.contiguous(), bn.weight, bn.bias, conv.weight, st, relu, int(conv.stride),
                           int(conv.padding), stats_out, defer)


def bn_fold_plan(x, cin, co1, k1, s1, p1, co2, k2, s2, p2) -> bool:
    """Whether conv1 (k1 x k1 / s1 / p1, cin -> co1) can emit the BatchNorm statistics of its output AND conv2
    (k2 / s2 / p2, co1 -> co2) can apply that BatchNorm in its A loader, for input ``x`` (NHWC) and the current
    micro-batch grouping (shape-only; cached by the caller)."""
    n, h, w = x.shape[0], x.shape[1], x.shape[2]
    return bool(_C().bn_fold_plan(n, h, w, x.shape[3], pad8(co1), k1, k1, s1, p1, pad8(co2), k2, k2, s2, p2,
                                  current_bn_groups()))


# ---------------------------------------------------------------------------------------------
# Pooling
# ---------------------------------------------------------------------------------------------
class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, relu):
        y, idx = _C().maxpool_fwd(x, k, s, p, relu)
        ctx.cfg = (x.shape[1], x.shape[2], k, s, p, relu)
        ctx.save_for_backward(y, idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, idx = ctx.saved_tensors
        h, w, k, s, p, relu = ctx.cfg
        return _C().maxpool_bwd(dy.contiguous(), y, idx, h, w, k, s, p, relu), None, None, None, None


def max_pool2d(x, kernel_size, stride=None, padding=0, relu=False):
    """Max pooling (optionally fused with a following ReLU: relu(maxpool(x)))."""
    stride = kernel_size if stride is None else stride
    if not x.is_cuda:
        y = F.max_pool2d(x, kernel_size, stride, padding)
        return F.relu(y) if relu else y
    return _MaxPoolFn.apply(x.contiguous(), int(kernel_size), int(stride), int(padding), relu)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[1], x.shape[2])
        return _C().avgpool_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return _C().avgpool_bwd(dy.contiguous(), *ctx.hw)


def global_avg_pool_flat(x):
    """AdaptiveAvgPool2d((1, 1)) + flatten -> [N, C]."""
    if not x.is_cuda:
        return _emu(torch.flatten(F.adaptive_avg_pool2d(x, (1, 1)), 1))
    return _AvgPoolFn.apply(x.contiguous())


def flatten_nchw(x, channels):
    """Flatten an activation in NCHW order ([N, C*H*W], the reference's ``x.view(-1, 320)``).
    GPU input is NHWC with padded channels; the real ``channels`` are kept."""
    if not x.is_cuda:
        return x.reshape(x.shape[0], -1)
    return x[..., :channels].permute(0, 3, 1, 2).reshape(x.shape[0], -1).contiguous()


# ---------------------------------------------------------------------------------------------
# Dropout
# ---------------------------------------------------------------------------------------------
class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, channel, salt):
        y, mask = _C().dropout_fwd(x, p, _rng_counter(x.device), salt, channel)
        ctx.p = p
        ctx.save_for_backward(mask)
        return y

    @staticmethod
    def backward(ctx, dy):
        (mask,) = ctx.saved_tensors
        return _C().dropout_bwd(dy.contiguous(), mask, ctx.p), None, None, None


_RNG: dict = {}
_SALT = [0]


def _rng_counter(device) -> torch.Tensor:
    """Per-device int64 RNG counter in device memory, seeded from torch's generator once and advanced by
    the dropout kernels themselves (so hipGraph replays draw new masks)."""
    key = (device.type, device.index)
    t = _RNG.get(key)
    if t is None:
        t = torch.randint(0, 2 ** 40, (1,), dtype=torch.long).to(device)
        _RNG[key] = t
    return t


def _seed() -> int:
    """Per-call-site salt (distinct streams for distinct dropout calls within a step)."""
    _SALT[0] = (_SALT[0] + 0x9E3779B97F4A7C15) % (2 ** 62)
    return _SALT[0]


def dropout(x, p=0.5, training=True, channel=False):
    """Dropout (``channel=True``: Dropout2d, one draw per (sample, channel))."""
    if not training or p == 0.0:
        return x
    if not x.is_cuda:
        return _emu(F.dropout2d(x, p, training) if channel else F.dropout(x, p, training))
    if x.dtype != torch.bfloat16:
        x = _C().cast_bf16(x.float().contiguous())
    return _DropoutFn.apply(x.contiguous(), float(p), channel, _seed())


# ---------------------------------------------------------------------------------------------
# Losses / log_softmax
# ---------------------------------------------------------------------------------------------
class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, mode):
        loss, lse = _C().ce_fwd(logits, target, mode)
        ctx.mode = mode
        ctx.out_f32 = logits.dtype == torch.float32
        ctx.save_for_backward(logits, target, lse)
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, target, lse = ctx.saved_tensors
        dx = _C().ce_bwd(logits, target, lse, g.float().contiguous().reshape(1), ctx.mode, ctx.out_f32)
        return dx, None, None


def cross_entropy(logits, target):
    """Mean cross-entropy (log_softmax + NLL fused)."""
    if not logits.is_cuda:
        return F.cross_entropy(logits.float(), target)
    return _CrossEntropyFn.apply(logits.contiguous(), target.contiguous(), 0)


def nll_loss(logp, target):
    """Mean NLL over log-probabilities."""
    if not logp.is_cuda:
        return F.nll_loss(logp, target)
    return _CrossEntropyFn.apply(logp.contiguous(), target.contiguous(), 1)


class _LogSoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = _C().log_softmax_fwd(x)
        ctx.in_f32 = x.dtype == torch.float32
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return _C().log_softmax_bwd(dy.float().contiguous(), y, ctx.in_f32)


def log_softmax(x, dim=1):
    if not x.is_cuda:
        return F.log_softmax(x, dim=dim)
    assert dim in (1, -1) and x.dim() == 2
    return _LogSoftmaxFn.apply(x.contiguous())


class _MSEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target):
        ctx.out_f32 = pred.dtype == torch.float32
        ctx.save_for_backward(pred, target)
        return _C().mse_fwd(pred, target)

    @staticmethod
    def backward(ctx, g):
        pred, target = ctx.saved_tensors
        return _C().mse_bwd(pred, target, g.float().contiguous().reshape(1), ctx.out_f32), None


def mse_loss(pred, target):
    if not pred.is_cuda:
        return F.mse_loss(pred.float(), target)
    return _MSEFn.apply(pred.contiguous(), target.float().contiguous())


# ---------------------------------------------------------------------------------------------
# EmbeddingBag (sum)
# ---------------------------------------------------------------------------------------------
class _EmbBagFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, indices, offsets):
        ctx.num = weight.shape[0]
        ctx.save_for_backward(indices, offsets)
        return _C().embbag_fwd(weight.detach().contiguous(), indices, offsets)

    @staticmethod
    def backward(ctx, dy):
        indices, offsets = ctx.saved_tensors
        return _C().embbag_bwd(dy.float().contiguous(), indices, offsets, ctx.num), None, None


def embedding_bag_sum(weight, indices, offsets):
    if not weight.is_cuda:
        return F.embedding_bag(indices, weight, offsets, mode="sum")
    return _EmbBagFn.apply(weight, indices.contiguous().long(), offsets.contiguous().long())


def kaiming_uniform_(t, a=math.sqrt(5)):
    return torch.nn.init.kaiming_uniform_(t, a=a)
