"""Multi-rank device path on one GPU, without PyTorch: 2, 4 or 8 processes each own a
wavelength slice (same device), join through the socket rendezvous (frei_amd.rendezvous) and exchange
the per-sweep partial sums either through the host hook or through the engine's P2P
mailboxes (IPC-mapped uncached device memory, per-value sequence flags, update kernel waits;
the same code path that runs over xGMI between GPUs).  Both must reproduce the single-rank
GPU run: identical T on every rank, the same convergence decision, T and spectrum within
the parity tolerance (only the bolometric summation order differs)."""
import multiprocessing as mp
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _problem():
    import frei_amd as fa
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), n_wl_bins=3001, n_layers=30, T_ref=2400)
    return grid, fa.load_example_opacity(grid, scale_factor=1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, transport, q):
    try:
        from frei_amd.distributed import host_comm, p2p_comm, partition
        from frei_amd.engine import Engine
        from frei_amd.rendezvous import Rendezvous
        rdzv = Rendezvous(world, rank, addr=("127.0.0.1", port), timeout=120)
        grid, op = _problem()
        lo, hi = partition(grid.lam.size, world, rank)
        comm = (p2p_comm if transport == "p2p" else host_comm)(rdzv)
        eng = Engine(grid.lam, grid.pressures, op, device=0, lam_slice=(lo, hi), comm=comm)
        out = eng.run(grid.init_temperatures, n_timesteps=60)
        # a second run on the same communicator (sequence numbers continue)
        out2 = eng.run(grid.init_temperatures, n_timesteps=60)
        chained = eng.chain_count()
        eng.close()
        rdzv.close()
        q.put((rank, lo, hi, out["spectrum"], out["final_T"], out["temp_hist"], out["n_iter"],
               out2["final_T"], None, chained))
    except Exception as e:   # reported to the parent, which fails the test
        q.put((rank, 0, 0, None, None, None, -1, None, repr(e), -1))


@pytest.mark.parametrize("transport,world", [("host", 2), ("p2p", 2), ("p2p", 4), ("host", 4),
                                             ("p2p", 8)])
def test_ranks_on_one_gpu_match_single_rank(transport, world):
    """world ranks (2, 4 and 8: the driver's 8-GPU layout, every mailbox fed by 7 peers)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, transport, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r[8] is None, f"rank {r[0]}: {r[8]}"
        # ranks sharing the GPU never chain launches (the runtime sees the peer mailboxes on its
        # own device): a chained launch's spinning sweep blocks could starve another rank
        assert r[9] == 0, f"rank {r[0]}: {r[9]} chained launches on a shared GPU"
    from frei_amd.engine import Engine
    grid, op = _problem()
    eng = Engine(grid.lam, grid.pressures, op, device=0)
    ref = eng.run(grid.init_temperatures, n_timesteps=60)
    eng.close()
    for r in res[1:]:
        assert np.array_equal(res[0][4], r[4])             # identical T on every rank
        assert r[6] == res[0][6]                           # same convergence decision
    assert np.array_equal(res[0][4], res[0][7])           # second run on the same comm
    assert res[0][6] == ref["n_iter"]
    assert np.max(np.abs(res[0][4] - ref["final_T"]) / ref["final_T"]) < 1e-11
    spec = np.concatenate([r[3] for r in res])
    assert np.max(np.abs(spec - ref["spectrum"]) / np.abs(ref["spectrum"])) < 1e-10


def _silent_worker(rank, world, port, q, hold_s):
    """Joins the P2P exchange (handles, mailbox mapping, handshake) and then never sweeps:
    a peer that stops publishing its sums.  Keeps its mailbox alive while the other rank
    runs into the timeout."""
    try:
        import time
        from frei_amd.distributed import p2p_comm, partition
        from frei_amd.engine import Engine
        from frei_amd.rendezvous import Rendezvous
        rdzv = Rendezvous(world, rank, addr=("127.0.0.1", port), timeout=120)
        grid, op = _problem()
        lo, hi = partition(grid.lam.size, world, rank)
        eng = Engine(grid.lam, grid.pressures, op, device=0, lam_slice=(lo, hi),
                     comm=p2p_comm(rdzv))
        rdzv.barrier()                    # both engines exist
        rdzv.barrier()                    # rank 0 has seen its error
        time.sleep(hold_s)
        eng.close()
        rdzv.close()
        q.put((rank, None))
    except Exception as e:
        q.put((rank, repr(e)))


def _timeout_worker(rank, world, port, q):
    try:
        import time
        from frei_amd.distributed import p2p_comm, partition
        from frei_amd.engine import Engine
        from frei_amd.rendezvous import Rendezvous
        rdzv = Rendezvous(world, rank, addr=("127.0.0.1", port), timeout=120)
        grid, op = _problem()
        lo, hi = partition(grid.lam.size, world, rank)
        eng = Engine(grid.lam, grid.pressures, op, device=0, lam_slice=(lo, hi),
                     comm=p2p_comm(rdzv))
        rdzv.barrier()
        t0 = time.monotonic()
        err = None
        try:
            eng.run(grid.init_temperatures, n_timesteps=20)
        except RuntimeError as e:
            err = str(e)
        dt = time.monotonic() - t0
        rdzv.barrier()
        eng.close()
        rdzv.close()
        q.put((rank, (err, dt)))
    except Exception as e:
        q.put((rank, repr(e)))


def test_p2p_missing_peer_fails_with_timeout_not_hang(monkeypatch):
    """A peer that joined the exchange but never publishes: the waiting rank's run ends with
    the engine's timeout error after about FREI_P2P_TIMEOUT_S (every later wait gives up at
    once), instead of hanging the GPU."""
    monkeypatch.setenv("FREI_P2P_TIMEOUT_S", "2")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_worker, args=(0, 2, port, q)),
             ctx.Process(target=_silent_worker, args=(1, 2, port, q, 1.0))]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None, res[1]
    err, dt = res[0]
    assert err is not None and "timed out" in err, res[0]
    assert dt < 60, dt
