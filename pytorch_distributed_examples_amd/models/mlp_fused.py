"""Fused training step for the elastic-DDP MLP (pytorch_elastic/mnist_ddp_elastic.py:133-173; the model of
:mod:`.mlp`), without autograd: one explicit launch sequence over preallocated activation buffers.

Per step, for L linear layers (7 for the reference 5x1024 model):

* 1 cast of the fp32 images into a bf16 activation buffer that carries a trailing ONES column;
* L forward GEMMs (bias + ReLU in the epilogue) writing straight into the next layer's padded buffer,
  whose ones column is set once at allocation;
* 1 fused cross-entropy launch: mean loss + d logits (bf16);
* L weight-gradient GEMMs that also produce the bias gradient: the GEMM runs over the input's ones
  column, and that output column (= the batch sum of dY) is routed to the bias gradient in the epilogue
  (``linear_wgrad_bias``) -- no column-sum kernel; weight and bias gradients land directly in the
  parameters' ``.grad`` (the DDP flat buffer), no zeroing, no accumulation copies;
* L-1 data-gradient GEMMs with the producer's ReLU mask applied in the epilogue (threshold_backward
  fused); the first layer's input gradient is never computed.  Each layer's dgrad and weight-gradient
  GEMMs go out as ONE paired launch (``OF.gemm_pair``), so the two small grids fill the chip together.

The layer-by-layer autograd path (``MLP.forward`` + ``backward()``) runs the same GEMMs plus autograd's
grad-zeroing, copies, casts and one bias column-sum per layer (≈60 launches per step vs ≈30 here).

    fmlp = FusedMLP(model)                       # model: MLP on the GPU
    ddp = DistributedDataParallel(model, overlap=False)
    loss = fmlp.forward_backward(x, y)           # grads written into p.grad (the DDP flat buffer)
    ddp.sync_gradients(); opt.step()
"""
from __future__ import annotations

import torch

from .. import _native
from ..ops import functional as OF
from ..ops import streams


def _pad8(n: int) -> int:
    return (n + 7) // 8 * 8


class FusedMLP:
    def __init__(self, net):
        self.net = net
        self.layers = [net.input_layer, *net.hidden_layers, net.final_layer]
        for i, L in enumerate(self.layers):
            assert L.bias is not None, "the fused step routes every bias gradient through the ones column"
            assert L.relu == (i < len(self.layers) - 1), "ReLU after every layer but the last"
        self._bufs: dict = {}

    def _buffers(self, B: int, dev: torch.device):
        key = (B, str(dev))
        if key not in self._bufs:
            bf = dict(dtype=torch.bfloat16, device=dev)
            acts = [torch.zeros(B, _pad8(self.layers[0].in_features + 1), **bf)]  # ones column: per-step cast
            for L in self.layers[:-1]:
                h = torch.zeros(B, _pad8(L.out_features + 1), **bf)
                h[:, L.out_features] = 1.0  # the GEMMs write [:, :out_features] only
                acts.append(h)
            logits = torch.empty(B, self.layers[-1].out_features, dtype=torch.float32, device=dev)
            dys = [torch.empty(B, L.out_features, **bf) for L in self.layers[:-1]]
            # d logits with its row padded to a multiple of 8 (zero columns, never written): the last layer's
            # dgrad then has K = 16 instead of 10 and runs on the FAST GEMM path with the zero-padded weight copy
            dlog = torch.zeros(B, _pad8(self.layers[-1].out_features), **bf)
            self._bufs[key] = (acts, logits, dys, dlog)
        return self._bufs[key]

    def _grads(self, L):
        for p in (L.weight, L.bias):
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        return L.weight.grad, L.bias.grad

    @torch.no_grad()
    def forward_backward(self, x: torch.Tensor, y: torch.Tensor, accumulate: bool = False, opt=None) -> torch.Tensor:
        """Mean cross-entropy of the batch (device scalar); parameter gradients written (``accumulate``:
        added) into each parameter's ``.grad``.

        ``opt`` (a fused optimiser, single process -- no gradient all-reduce between backward and update):
        the optimiser step is folded into the backward: layer i+1's update runs as extra blocks of layer i's
        paired dgrad + wgrad launch (its gradients are final by then, and no GEMM of that launch touches its
        weights), layers 1 and 0 in one closing launch.  Replaces ``opt.step()``; same update math, same
        kernels' device code."""
        C = _native.C()
        params_of = [[L.weight, L.bias] for L in self.layers]
        fuse_opt = (opt is not None and not streams.active_for(x) and
                    opt.supports_segments([p for ps in params_of for p in ps]))
        if fuse_opt:
            for L in self.layers:  # every gradient exists up front: ONE optimiser table for the whole step
                self._grads(L)
        B = x.shape[0]
        acts, logits, dys, dlog = self._buffers(B, x.device)
        C.cast_rows_ones(x.reshape(B, -1).float().contiguous(), acts[0])
        last = len(self.layers) - 1
        for i, L in enumerate(self.layers):
            w = OF._bf16_weight(L.weight)
            out = acts[i + 1][:, :L.out_features] if i < last else logits
            C.linear_fwd_out(acts[i][:, :L.in_features], w, L.bias.detach(), i < last, out)
        nout = self.layers[-1].out_features
        loss, dy = C.ce_fused(logits, y.long().contiguous(), dlog)
        dy = dlog[:, :nout]
        side = streams.active_for(x)
        for i in range(last, -1, -1):
            L = self.layers[i]
            gw, gb = self._grads(L)
            if side:
                # (opt-in, ops/streams.py) weight + bias gradient on the side stream, concurrent with the dgrad
                # chain (forked before the dgrad is enqueued so the fork point does not wait for it)
                with streams.fork(dy, join_at_backward_end=False):
                    C.linear_wgrad_bias(dy, acts[i][:, :L.in_features + 1], gw, gb, accumulate)
            elif i > 0:
                # dgrad + weight/bias gradient as ONE paired GEMM launch (dgrad tiles first), carrying the update
                # of layer i + 1 when the optimiser is folded in
                wpad = OF._maintained(L.weight, "bf16_pad") if i == last else None
                if fuse_opt and i < last:
                    opt.attach_update(params_of[i + 1])
                with OF.gemm_pair(defer_second=True, flush_by_caller=True):
                    if wpad is not None:  # K padded to 16: zero columns of d logits x zero rows of the weight
                        C.linear_dgrad_out(dlog, wpad, acts[i][:, :L.in_features], dys[i - 1])
                    else:
                        C.linear_dgrad_out(dy, OF._bf16_weight(L.weight), acts[i][:, :L.in_features], dys[i - 1])
                    C.linear_wgrad_bias(dy, acts[i][:, :L.in_features + 1], gw, gb, accumulate)
                dy = dys[i - 1]
                continue
            else:
                C.linear_wgrad_bias(dy, acts[i][:, :L.in_features + 1], gw, gb, accumulate)
            if i > 0:
                C.linear_dgrad_out(dy, OF._bf16_weight(L.weight), acts[i][:, :L.in_features], dys[i - 1])
                dy = dys[i - 1]
        # the deferred weight-gradient reductions: one batched launch (and the side stream, if used)
        streams.join(x.device)
        if fuse_opt:  # the updates no backward launch could carry: layers 0 and 1 (1 only if it exists)
            opt.step_range([p for ps in params_of[:min(2, last + 1)] for p in ps], last=True)
        return loss

    def launches_per_step(self) -> int:
        """Kernel launches of one forward_backward (split-K GEMMs add their reduce launch on top)."""
        n = len(self.layers)
        return 1 + n + 1 + n + (n - 1)
