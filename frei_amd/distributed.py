"""Wavelength sharding across GPUs.

One process per GPU; each owns the contiguous slice ``partition(n_lam, nranks, rank)``
of the global grid.  Bolometric sums use per-point trapezoid weights of the GLOBAL grid,
so a slice needs no halo; the only exchange is one all-gather of the per-sweep partial
sums (n_layers x 4 doubles), summed in rank order on every rank (bitwise-identical T).

Transports: RCCL over xGMI inside the native engine (``rccl_comm``), or a host
all-gather through torch.distributed/gloo (``gloo_comm``) for ranks sharing a GPU.
"""
import ctypes

import numpy as np

from . import _native as N
from .engine import partition

__all__ = ["partition", "rccl_comm", "gloo_comm"]


def rccl_comm(dist, nranks, rank):
    """RCCL communicator spec for Engine(comm=...): rank 0 creates the unique id and
    ``dist`` (an initialised torch.distributed) broadcasts it."""
    uid = None
    if rank == 0:
        buf = ctypes.create_string_buffer(128)
        N.check(N.lib().frei_comm_unique_id(buf))
        uid = buf.raw
    obj = [uid]
    dist.broadcast_object_list(obj, src=0)
    return ("rccl", nranks, rank, obj[0])


def gloo_comm(dist, nranks, rank):
    """Host all-gather spec (torch.distributed CPU tensors)."""
    import torch

    def allgather(send):
        t = torch.from_numpy(np.ascontiguousarray(send))
        out = [torch.empty_like(t) for _ in range(nranks)]
        dist.all_gather(out, t)
        return np.concatenate([o.numpy() for o in out])
    return ("host", nranks, rank, allgather)
