"""Multi-GPU launch helpers for the partitioned solver.

One process per GPU, launched by torch.distributed.run; torch.distributed is used only as the
rendezvous (and, for the test transport, as the reducer) -- the solver's per-iteration
all-reduces run on RCCL inside libaa_admm.so, enqueued on the solver's HIP stream.
"""
from __future__ import annotations

import numpy as np

from . import capi


def rccl_comm(ctx: capi.Context, rank: int, size: int, group=None) -> capi.Comm:
    """RCCL communicator over xGMI: rank 0 creates the unique id, torch.distributed broadcasts it."""
    if size == 1:
        return capi.Comm.rccl(ctx, 0, 1, capi.Comm.unique_id())
    import torch.distributed as dist
    obj = [capi.Comm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return capi.Comm.rccl(ctx, rank, size, obj[0])


def host_comm(rank: int, size: int, group=None) -> capi.Comm:
    """Host-staged transport over torch.distributed (gloo): SUM then a broadcast from rank 0,
    so every rank receives bit-identical values whatever the backend's reduction order."""
    if size == 1:
        return capi.Comm.host(lambda a: None, 0, 1)
    import torch
    import torch.distributed as dist

    def reduce(a: np.ndarray):
        t = torch.from_numpy(a)   # shares memory with the C buffer
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        dist.broadcast(t, src=0, group=group)

    return capi.Comm.host(reduce, rank, size)
