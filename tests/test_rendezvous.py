"""The socket rendezvous of the multi-rank path (frei_amd.rendezvous; no PyTorch): all-gather
in rank order, broadcast, barrier and max over 3 processes, with an explicit address and with
the launcher-style discovery (rank 0 publishes an ephemeral port in a file keyed by the
launch)."""
import multiprocessing as mp
import socket
import struct

import pytest

from frei_amd.rendezvous import Rendezvous


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, addr, tag, q):
    r = Rendezvous(world, rank, addr=addr, tag=tag, timeout=60)
    got = r.all_gather(struct.pack("!i", 10 * rank + 1))
    r.barrier()
    b = r.broadcast(b"hello" if rank == 1 else b"", src=1)
    m = r.max(float(rank) * 1.5)
    big = r.all_gather(bytes([rank]) * (1 << 20))     # 1 MiB per rank
    r.close()
    q.put((rank, [struct.unpack("!i", x)[0] for x in got], b, m, [len(x) for x in big],
           [x[0] for x in big]))


@pytest.mark.parametrize("mode", ["addr", "file"])
def test_rendezvous_collectives(mode, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 3
    addr = ("127.0.0.1", _free_port()) if mode == "addr" else None
    tag = None if mode == "addr" else f"test-{tmp_path.name}"
    ps = [ctx.Process(target=_worker, args=(r, world, addr, tag, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps])
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, got, b, m, sizes, first in res:
        assert got == [1, 11, 21]              # rank order on every rank
        assert b == b"hello"
        assert m == 3.0
        assert sizes == [1 << 20] * world and first == [0, 1, 2]


def test_single_rank_is_local():
    r = Rendezvous(1, 0)
    assert r.all_gather(b"x") == [b"x"]
    assert r.max(2.5) == 2.5
    r.barrier()
