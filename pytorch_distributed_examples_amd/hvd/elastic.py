"""Horovod-elastic API: ``run``, ``State``, ``ObjectState``, ``TorchState`` (horovod/torch/elastic).

Used by the reference at horovod/horovod_mnist_elastic.py:55,72,80-82,104-106.

* ``TorchState(model, optimizer, **kw)`` keeps an in-memory commit of the model/optimizer state dicts and
  the extra attributes (``batch``, ``epoch``).  Commits are DEVICE-resident clones (an MI355X has 288 GB
  of HBM; a clone is one D2D copy instead of a PCIe round trip) -- ``restore()`` copies them back.
* ``commit()`` = ``core.check_health()`` (a timed-out xGMI exchange inside a replayed graph raises
  :class:`HorovodInternalError` BEFORE the suspect state is saved) + ``save()`` + ``check_host_updates()``
  (raises :class:`HostsUpdatedInterrupt` when the elastic driver published a membership change).
* ``sync()`` broadcasts the state from the new rank 0 (always a survivor holding the latest commit).
* Failures are TYPED at their source (no message matching): the engine, ``core.check_health()`` and every
  gloo control-plane call (``core._control_plane``) raise :class:`HorovodInternalError`; any other exception
  is a bug and propagates.
* ``@run`` retries ``func(state)``: on :class:`HorovodInternalError` (a peer died mid-collective) it
  restores the last commit; on ``HostsUpdatedInterrupt`` it keeps the state; both then ``reset()``:
  in-process ``shutdown()`` + ``init()`` into the driver's next rendezvous round (new process group, new
  RCCL communicator) followed by the reset callbacks (e.g. the LR rescale of horovod_mnist_elastic.py:80).
"""
from __future__ import annotations

import copy
import functools

import torch

from . import core
from ..utils.state import clone_state as _clone
from .exceptions import HorovodInternalError, HostsUpdatedInterrupt
from .functions import broadcast_optimizer_state, broadcast_parameters


class State:
    def __init__(self):
        self._reset_callbacks = []

    def register_reset_callbacks(self, callbacks):
        self._reset_callbacks.extend(callbacks)

    def on_reset(self):
        self._host_messages_checked = True
        for cb in self._reset_callbacks:
            cb()

    def commit(self):
        core.check_health()
        self.save()
        self.check_host_updates()

    def check_host_updates(self):
        rd = core._ctx.rdzv
        if rd is None:
            return
        updated = rd.hosts_updated()
        # every rank must agree (a rank that saw the flag late would otherwise keep training alone)
        # gloo control plane (host tensor): a dead peer is a connection error here, not a hung GPU collective
        flag = torch.tensor([1.0 if updated else 0.0])
        with core._control_plane("check_host_updates"):  # a dead peer surfaces here, typed
            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MAX, group=core._ctx.group)
        if flag.item() > 0:
            raise HostsUpdatedInterrupt(skip_sync=False)

    def save(self):
        raise NotImplementedError

    def restore(self):
        raise NotImplementedError

    def sync(self):
        raise NotImplementedError

    def reset(self):
        pass


class ObjectState(State):
    """Arbitrary picklable attributes, synchronised with ``broadcast_object``."""

    def __init__(self, bcast_object=None, **kwargs):
        super().__init__()
        self._bcast_object = bcast_object or core.broadcast_object
        self._saved_state = dict(kwargs)
        for k, v in kwargs.items():
            setattr(self, k, v)

    def save(self):
        self._saved_state = {k: copy.deepcopy(getattr(self, k)) for k in self._saved_state}

    def restore(self):
        for k, v in self._saved_state.items():
            setattr(self, k, copy.deepcopy(v))

    def sync(self):
        if self._saved_state:
            self._saved_state = self._bcast_object(self._saved_state)
            ObjectState.restore(self)  # attributes only (a subclass restore would roll back tensors)


class TorchState(ObjectState):
    def __init__(self, model=None, optimizer=None, **kwargs):
        self.model = model
        self.optimizer = optimizer
        self._saved_model_state = None
        self._saved_optimizer_state = None
        super().__init__(bcast_object=None, **kwargs)
        self.save()

    def save(self):
        if self.model is not None:
            self._saved_model_state = _clone(self.model.state_dict())
        if self.optimizer is not None:
            self._saved_optimizer_state = _clone(self.optimizer.state_dict())
        super().save()

    def restore(self):
        if self.model is not None and self._saved_model_state is not None:
            self.model.load_state_dict(self._saved_model_state)
        if self.optimizer is not None and self._saved_optimizer_state is not None:
            self.optimizer.load_state_dict(_clone(self._saved_optimizer_state))
        super().restore()

    def sync(self):
        if self.model is not None:
            broadcast_parameters(self.model.state_dict(), root_rank=0)
        if self.optimizer is not None:
            broadcast_optimizer_state(self.optimizer, root_rank=0)
        super().sync()


def reset():
    """In-process re-rendezvous: tear down comm state and join the driver's next round."""
    core.shutdown(abort=True)
    core.init()


def run(func):
    """Decorator for the elastic training function ``func(state, *args, **kwargs)``."""

    @functools.wraps(func)
    def wrapper(state, *args, **kwargs):
        skip_sync = False
        while True:
            try:
                if not skip_sync:
                    state.sync()
                return func(state, *args, **kwargs)
            except HorovodInternalError:
                state.restore()
                skip_sync = False
            except HostsUpdatedInterrupt as e:
                skip_sync = e.skip_sync
            reset()
            state.on_reset()

    return wrapper
