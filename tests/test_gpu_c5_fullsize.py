"""Config C5 at its real per-atmosphere size against the oracle (VERDICT r03 "next" #6).

C5 is a grid sweep of atmospheres over T_ref x log g x [M/H]; bench.py runs
32 of them per GPU as one batched context: 60 layers x 100k λ x 8 species each, the species
contraction per atmosphere on fp64 MFMA (K7), sweeps over (λ block, atmosphere).  Here four
corners of that grid — T_ref 1000 / 2400 K, log g 2.5 / 4, [M/H] -1 / +1 — run batched at full
size with bench.py's tables (c5_leg), a fixed 3 T-P iterations plus the final emit, and every
atmosphere is compared with the oracle run on that atmosphere alone (the reference's per-Grid
loop, core.py:233-338), λ-sharded over worker processes (oracle/sharded.py).  Criterion:
tests/parity.py assert_grid_parity (1e-10, or twice the one-ulp floor of the reference
algorithm measured on the same inputs), T within 1e-10; the errors go to the parity log.
"""
import numpy as np
import pytest

from tests.parity import assert_grid_parity, grid_floor
from oracle.sharded import ShardedOracle

pytestmark = pytest.mark.gpu

M_BAR = 4.0142926168559996e-24
FIXED = dict(n_timesteps=3, n_zero_crossings=10 ** 6, convergence_dT=-1.0)


def test_c5_batched_atmospheres_match_oracle_at_full_size():
    import frei_amd as fa
    from frei_amd.batch import BatchEngine
    from frei_amd.opacity import SeparableTable
    from frei_amd.tp import temperature_grid
    from frei_amd.workloads import c3
    w = c3(n_layers=60, n_lam=100_000, n_T=16)
    corners = [(1000.0, 2.5, -1.0), (2400.0, 4.0, 1.0), (1000.0, 4.0, 1.0), (2400.0, 2.5, -1.0)]
    T0 = np.array([temperature_grid(w["p"], t, 0.1, 0.1) for t, _, _ in corners])
    g = np.array([10.0 ** lg for _, lg, _ in corners])
    T_nodes = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 16)    # bench.py c5_leg's nodes
    fT = (T_nodes / 1000.0) ** 0.5
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], fT, w["p"], T_nodes)
            for s, n in enumerate(w["names"])}
    mmr = np.array([w["mmr"] * 10.0 ** mh for _, _, mh in corners])
    eng = BatchEngine(w["lam"], w["p"], tabs, g=g, mmr=mmr)
    try:
        assert eng.path()["contracted"]          # K7: per-atmosphere contraction (MFMA)
        out = eng.run(T0, alpha=1.0, **FIXED)
        ups, downs = eng.get_fluxes()
    finally:
        eng.close()
    assert list(out["n_iter"]) == [3] * len(corners)
    o_tabs = {n: (w["base"][s], w["fp"][s], fT, T_nodes) for s, n in enumerate(w["names"])}
    Ft = fa.F_TOA(w["lam"])
    for m, (t_ref, lg, mh) in enumerate(corners):
        with ShardedOracle(o_tabs, w["lam"], w["p"], T0[m], Ft, g[m], M_BAR,
                           mmr=mmr[m]) as so:
            o = so.emission_spectrum(**FIXED)
            pt = so.emission_spectrum(perturb=True, **FIXED)
        assert o[6] == 3
        floor = grid_floor(o[0], o[4], o[5], pt[0], pt[4], pt[5])
        assert_grid_parity(out["spectra"][m], o[0], ups[m], o[4], downs[m], o[5],
                           f"C5 60x100000x8 atmosphere T_ref {t_ref:.0f} log g {lg} "
                           f"[M/H] {mh:+.0f}", floor, T=out["final_T"][m], ref_T=o[1])
