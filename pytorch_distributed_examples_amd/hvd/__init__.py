"""Horovod-compatible API (``import pytorch_distributed_examples_amd.hvd as hvd``) on the MI355X runtime.

Drop-in for the subset of ``horovod.torch`` the reference uses (horovod/mnist_horovod.py,
horovod/horovod_mnist_elastic.py) plus the rest of the common surface: init/shutdown/size/rank/
local_rank/local_size/cross_rank, allreduce(+_/async), grouped_allreduce, allgather, broadcast(+_/async),
alltoall, synchronize/poll/join/barrier, broadcast_object/allgather_object, broadcast_parameters,
broadcast_optimizer_state, DistributedOptimizer, Compression, ReduceOp (Average/Sum/Min/Max/Product),
and ``hvd.elastic`` (run, State, ObjectState, TorchState).  Backed by the C++ fusion engine and an RCCL
communicator of our own (csrc/comm) -- see :mod:`.core`.
"""
from . import elastic
from .core import (Adasum, Average, Max, Min, Product, ReduceOp, Sum, allgather, allgather_async, allgather_object,
                   allreduce, allreduce_, allreduce_async, allreduce_async_, alltoall, barrier, broadcast, broadcast_,
                   broadcast_async, broadcast_async_, broadcast_object, cross_rank, cross_size, engine_stats,
                   gloo_built, gpu_available, grouped_allreduce, init, is_homogeneous, is_initialized, join,
                   local_rank, local_size, mpi_built, nccl_built, poll, rank, rocm_built, shutdown, size, synchronize)
from .exceptions import HorovodInternalError, HostsUpdatedInterrupt
from .functions import broadcast_optimizer_state, broadcast_parameters
from .optimizer import Compression, DistributedOptimizer

__all__ = [n for n in dir() if not n.startswith("_")]
