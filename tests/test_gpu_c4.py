"""Config C4: the full C3 workload — 60 layers x 500k wavelengths x 8
species (6 molecules + 2 CIA tables) — run to radiative equilibrium with the reference's
convergence test (n_zero_crossings = 2, convergence_dT = 3 K; core.py:273-318), four ways:

- unsharded, species contraction (K3) — the benchmark's path;
- unsharded, per-species sum in the sweep (``precontract`` off);
- two ranks, each owning half of the wavelengths, exchanging through the host hook;
- two ranks exchanging through the engine's P2P mailboxes (the multi-GPU path).

The oracle cannot follow 500k wavelengths to convergence in test time, so the checks are the
size-independent ones: identical iteration counts, bitwise-identical temperatures on every
rank, temperatures within 1e-12 of the unsharded run (only the bolometric summation tree
differs) and within 1e-10 for the per-species path (the species sum is reordered), and the
sharded spectra reassembling the unsharded one.
"""
import multiprocessing as mp
import socket

import numpy as np
import pytest

from tests.parity import rel

pytestmark = pytest.mark.gpu

RUN = dict(n_timesteps=200, n_zero_crossings=2, convergence_dT=3.0, want_dtaus=False)


def _tables():
    import frei_amd as fa
    from frei_amd.workloads import c3
    w = c3()
    tabs = {n: fa.SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, n in enumerate(w["names"])}
    return w, tabs


def _chem(fa, w):
    """T-dependent chemistry for the C3 species (frei_amd.workloads.c3_chemistry), re-interpolated
    on the device before every sweep; the sweep keeps the per-species sum."""
    from frei_amd.workloads import c3_chemistry
    return c3_chemistry(w)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, transport, q, chem=False):
    try:
        from frei_amd.distributed import host_comm, p2p_comm, partition
        from frei_amd.engine import Engine
        from frei_amd.rendezvous import Rendezvous
        rdzv = Rendezvous(world, rank, addr=("127.0.0.1", port), timeout=180)
        w, tabs = _tables()
        lo, hi = partition(w["lam"].size, world, rank)
        comm = (p2p_comm if transport == "p2p" else host_comm)(rdzv)
        if chem:
            import frei_amd as fa
            mmr = _chem(fa, w)
        else:
            mmr = w["mmr"]
        eng = Engine(w["lam"], w["p"], tabs, mmr=mmr, device=0, lam_slice=(lo, hi),
                     comm=comm)
        out = eng.run(w["T0"], **RUN)
        eng.close()
        rdzv.close()
        q.put((rank, lo, hi, out["n_iter"], out["final_T"], out["spectrum"], None))
    except Exception as e:
        q.put((rank, 0, 0, -1, None, None, repr(e)))


@pytest.fixture(scope="module")
def unsharded():
    from frei_amd.engine import Engine
    w, tabs = _tables()
    out = {}
    eng = Engine(w["lam"], w["p"], tabs, mmr=w["mmr"])
    try:
        for mode, opt in (("contracted", -1), ("per_species", 0)):
            eng.set_option("precontract", opt)
            assert eng.path()["contracted"] == (mode == "contracted")
            out[mode] = eng.run(w["T0"], **RUN)
    finally:
        eng.close()
    return w, out


def test_c4_contracted_and_per_species_converge_alike(unsharded):
    w, out = unsharded
    a, b = out["contracted"], out["per_species"]
    assert 1 < a["n_iter"] < RUN["n_timesteps"], a["n_iter"]   # converged, not capped
    assert a["n_iter"] == b["n_iter"]
    assert rel(b["final_T"], a["final_T"]) < 1e-10
    assert rel(b["spectrum"], a["spectrum"]) < 1e-9
    assert np.isfinite(a["spectrum"]).all() and (a["spectrum"] > 0).all()
    assert rel(a["final_T"], w["T0"]) > 1e-3      # the profile moved toward equilibrium


@pytest.mark.parametrize("transport", ["host", "p2p"])
def test_c4_two_rank_lambda_shards_match_unsharded(unsharded, transport):
    w, out = unsharded
    ref = out["contracted"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, transport, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r[6] is None, f"rank {r[0]}: {r[6]}"
    assert res[0][3] == res[1][3] == ref["n_iter"]
    assert np.array_equal(res[0][4], res[1][4])            # bitwise-identical T on every rank
    assert rel(res[0][4], ref["final_T"]) < 1e-12
    assert res[0][2] == res[1][1] and res[1][2] == w["lam"].size
    spec = np.concatenate([res[0][5], res[1][5]])
    assert rel(spec, ref["spectrum"]) < 1e-10


def test_c4_chemistry_two_rank_p2p_matches_unsharded():
    """C4 with T-dependent chemistry: the per-species sweep with mixing ratios re-evaluated
    at every layer's current T each sweep, to convergence, unsharded and as two P2P ranks."""
    import frei_amd as fa
    from frei_amd.engine import Engine
    w, tabs = _tables()
    eng = Engine(w["lam"], w["p"], tabs, mmr=_chem(fa, w))
    try:
        assert not eng.path()["contracted"]
        ref = eng.run(w["T0"], **RUN)
    finally:
        eng.close()
    assert 1 < ref["n_iter"] < RUN["n_timesteps"], ref["n_iter"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, "p2p", q, True)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r[6] is None, f"rank {r[0]}: {r[6]}"
    assert res[0][3] == res[1][3] == ref["n_iter"]
    assert np.array_equal(res[0][4], res[1][4])
    assert rel(res[0][4], ref["final_T"]) < 1e-12
    spec = np.concatenate([res[0][5], res[1][5]])
    assert rel(spec, ref["spectrum"]) < 1e-10
