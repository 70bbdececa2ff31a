"""Wavelength sharding across GPUs.

One process per GPU; each owns the contiguous slice ``partition(n_lam, nranks, rank)``
of the global grid.  Bolometric sums use per-point trapezoid weights of the GLOBAL grid,
so a slice needs no halo; the only exchange is the per-sweep partial sums (n_layers x 4
doubles), summed in rank order on every rank (bitwise-identical T).

Transports (``Engine(comm=...)``), all set up through a plain-socket
:class:`~frei_amd.rendezvous.Rendezvous` (no PyTorch anywhere on this path):
- ``p2p_comm``: the engine's own device-resident exchange over xGMI — every rank pushes its
  sums into every rank's IPC-mapped mailbox, the update kernel waits on per-value flags;
- ``rccl_comm``: one ``ncclAllGather`` per sweep inside the engine (RCCL, dlopen'ed);
- ``host_comm``: the per-sweep all-gather through the host (tests; ranks sharing a GPU).
"""
import ctypes

import numpy as np

from . import _native as N
from .engine import partition
from .rendezvous import Rendezvous, from_env

__all__ = ["partition", "p2p_comm", "rccl_comm", "host_comm", "Rendezvous", "from_env"]


def p2p_comm(rdzv):
    """P2P mailbox spec for Engine(comm=...): the IPC handles are all-gathered through
    ``rdzv`` once, when the engine joins."""
    return ("p2p", rdzv.world, rdzv.rank, rdzv.all_gather)


def rccl_comm(rdzv):
    """RCCL communicator spec: rank 0 creates the unique id, ``rdzv`` broadcasts it."""
    uid = b""
    if rdzv.rank == 0:
        buf = ctypes.create_string_buffer(128)
        N.check(N.lib().frei_comm_unique_id(buf))
        uid = buf.raw
    return ("rccl", rdzv.world, rdzv.rank, rdzv.broadcast(uid, src=0))


def host_comm(rdzv):
    """Host all-gather spec: every sweep's partial sums go through ``rdzv`` (rank order)."""
    def allgather(send):
        parts = rdzv.all_gather(np.ascontiguousarray(send, dtype=np.float64).tobytes())
        return np.concatenate([np.frombuffer(p, dtype=np.float64) for p in parts])
    return ("host", rdzv.world, rdzv.rank, allgather)
