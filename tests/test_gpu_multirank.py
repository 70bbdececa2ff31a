"""Multi-rank device path on one GPU: two processes each own a wavelength slice (same
device), exchange per-sweep partial sums through the C ABI's host all-gather hook
(gloo), and must reproduce the single-rank GPU run.  (RCCL refuses two ranks on one
device; the RCCL transport differs only in how the same n_layers*4 doubles move.)"""
import os
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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from frei_amd.distributed import gloo_comm, partition
    from frei_amd.engine import Engine
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grid, op = _problem()
    lo, hi = partition(grid.lam.size, world, rank)
    eng = Engine(grid.lam, grid.pressures, op, device=0, lam_slice=(lo, hi),
                 comm=gloo_comm(dist, world, rank))
    out = eng.run(grid.init_temperatures, n_timesteps=60)
    q.put((rank, lo, hi, out["spectrum"], out["final_T"], out["temp_hist"], out["n_iter"]))
    eng.close()
    dist.destroy_process_group()


def test_two_ranks_one_gpu_match_single_rank():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from frei_amd.engine import Engine
    grid, op = _problem()
    eng = Engine(grid.lam, grid.pressures, op, device=0)
    ref = eng.run(grid.init_temperatures, n_timesteps=60)
    eng.close()
    assert np.array_equal(res[0][4], res[1][4])           # identical T on every rank
    assert res[0][6] == res[1][6] == ref["n_iter"]         # same convergence decision
    assert np.max(np.abs(res[0][4] - ref["final_T"]) / ref["final_T"]) < 1e-11
    spec = np.concatenate([r[3] for r in res])
    assert np.max(np.abs(spec - ref["spectrum"]) / np.abs(ref["spectrum"])) < 1e-9
