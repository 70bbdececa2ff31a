"""Process-group plumbing for one-process-per-GPU runs, in plain sockets (no PyTorch).

The multi-GPU path needs a handful of host-side collectives, none of them on the data path:
exchanging the RCCL unique id or the P2P mailbox IPC handles once, barriers and the
max-over-ranks of wall-clock timings in ``bench.py``, and (for ranks that share one GPU in
tests) the host all-gather of the per-sweep bolometric partial sums.  :class:`Rendezvous` is a
star over TCP on 127.0.0.1: rank 0 accepts one connection per peer; ``all_gather`` sends
every rank's bytes to rank 0, which returns the rank-ordered list to everyone.

Discovery (single node, as the driver launches ``torch.distributed.run --nnodes=1``):
- ``addr=(host, port)`` given: rank 0 listens there;
- otherwise rank 0 binds an ephemeral port on 127.0.0.1 and publishes it in a file named by
  ``MASTER_PORT`` and the parent process id (every rank of one launch shares the launcher
  as parent), so it never competes with the launcher's own store on ``MASTER_PORT``.
"""
import os
import socket
import struct
import tempfile
import time

__all__ = ["Rendezvous", "from_env"]

_HDR = struct.Struct("!q")


def _send(sock, b):
    sock.sendall(_HDR.pack(len(b)) + b)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock):
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return _recv_exact(sock, n)


def _read_port(path):
    """("127.0.0.1", port) from rank 0's port file, or None while it is absent / half written."""
    try:
        with open(path) as f:
            txt = f.read().strip()
        return ("127.0.0.1", int(txt)) if txt else None
    except (OSError, ValueError):
        return None


class Rendezvous:
    """``world`` ranks, this one ``rank``; see the module docstring for discovery."""

    def __init__(self, world, rank, addr=None, timeout=120.0, tag=None):
        if not (0 <= rank < world):
            raise ValueError("bad rank / world size")
        self.world, self.rank = int(world), int(rank)
        self._peers = []          # rank 0: sockets of ranks 1..world-1, in rank order
        self._sock = None         # rank > 0: socket to rank 0
        self._file = None
        if self.world == 1:
            return
        deadline = time.monotonic() + timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind(addr if addr is not None else ("127.0.0.1", 0))
            srv.listen(self.world)
            if addr is None:
                self._file = _port_file(tag)
                tmp = self._file + ".tmp"
                with open(tmp, "w") as f:
                    f.write(str(srv.getsockname()[1]))
                os.replace(tmp, self._file)
            srv.settimeout(max(1.0, deadline - time.monotonic()))
            by_rank = {}
            try:
                while len(by_rank) < self.world - 1:
                    conn, _ = srv.accept()
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    conn.settimeout(None)
                    (r,) = struct.unpack("!i", _recv_exact(conn, 4))
                    by_rank[r] = conn
            finally:
                srv.close()
                if self._file is not None:
                    try:
                        os.unlink(self._file)
                    except OSError:
                        pass
            self._peers = [by_rank[r] for r in range(1, self.world)]
        else:
            path = _port_file(tag) if addr is None else None
            while True:
                # the port file is re-read before every attempt: a stale file left by a crashed
                # earlier launch with the same key is replaced when rank 0 publishes its port
                target = addr if path is None else _read_port(path)
                try:
                    if target is None:
                        raise OSError("port not published yet")
                    s = socket.create_connection(target, timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        if target is None:
                            raise TimeoutError(f"rendezvous: rank 0 never published {path}")
                        raise
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(None)
            s.sendall(struct.pack("!i", self.rank))
            self._sock = s

    # ------------------------------------------------------------------ collectives
    def all_gather(self, b):
        """Every rank's ``bytes`` in rank order, on every rank."""
        b = bytes(b)
        if self.world == 1:
            return [b]
        if self.rank == 0:
            out = [b] + [_recv(p) for p in self._peers]
            packed = b"".join(_HDR.pack(len(x)) + x for x in out)
            for p in self._peers:
                _send(p, packed)
            return out
        _send(self._sock, b)
        packed = _recv(self._sock)
        out, off = [], 0
        for _ in range(self.world):
            (n,) = _HDR.unpack_from(packed, off)
            off += _HDR.size
            out.append(packed[off:off + n])
            off += n
        return out

    def barrier(self):
        self.all_gather(b"")

    def broadcast(self, b, src=0):
        return self.all_gather(b if self.rank == src else b"")[src]

    def max(self, x):
        vals = self.all_gather(struct.pack("!d", float(x)))
        return max(struct.unpack("!d", v)[0] for v in vals)

    def close(self):
        for s in self._peers:
            s.close()
        self._peers = []
        if self._sock is not None:
            self._sock.close()
            self._sock = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _port_file(tag):
    tag = tag or f"{os.environ.get('MASTER_PORT', '0')}-{os.getppid()}"
    return os.path.join(tempfile.gettempdir(), f"frei-rdzv-{tag}.port")


def from_env(timeout=120.0):
    """Rendezvous of a ``torch.distributed.run``-style launch (WORLD_SIZE / RANK in the
    environment; the launcher itself is not otherwise used)."""
    return Rendezvous(int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
                      timeout=timeout)
