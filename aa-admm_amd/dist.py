"""Multi-GPU launch helpers for the partitioned solver.

One process per GPU, launched by torch.distributed.run, which is only the launcher: the rank
processes never import torch (rdzv.py says why) and rendezvous through `rdzv.Group` -- the RCCL
unique id, barriers, timing reductions and the host transport. The solver's per-iteration
all-reduces run on RCCL inside libaa_admm.so, enqueued on the solver's HIP stream.

`rank_setup()` is the first thing a rank process does: it loads libaa_admm.so, checks that the
process is bound to the ROCm runtime the library was built against (capi.check_runtime) and
joins the group.
"""
from __future__ import annotations

import numpy as np

from . import capi
from .rdzv import Group


def rank_setup(timeout: float = 600.0):
    """(group, runtime report) of this rank: library loaded and its runtime checked BEFORE the
    rendezvous, so a mis-bound rank fails before any rank touches a GPU."""
    capi.lib()
    report = capi.check_runtime()
    return Group.from_env(timeout), report


def rccl_comm(ctx: capi.Context, group: Group) -> capi.Comm:
    """RCCL communicator over xGMI: rank 0 creates the unique id, the group broadcasts it."""
    if group.size == 1:
        return capi.Comm.rccl(ctx, 0, 1, capi.Comm.unique_id())
    uid = group.broadcast_bytes(capi.Comm.unique_id() if group.rank == 0 else None)
    return capi.Comm.rccl(ctx, group.rank, group.size, uid)


def host_comm(group: Group) -> capi.Comm:
    """Host-staged transport over the group: rank-order SUM at rank 0, the same bits returned to
    every rank (lets several ranks share one GPU)."""
    if group.size == 1:
        return capi.Comm.host(lambda a: None, 0, 1)

    def reduce(a: np.ndarray):
        group.allreduce_array(a, "sum")   # a shares memory with the C buffer

    return capi.Comm.host(reduce, group.rank, group.size)
