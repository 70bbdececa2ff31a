"""Radiative equilibrium at BASELINE size against the oracle (VERDICT r03 "next" #1).

BASELINE.json's metric has two halves: flux updates/s and "T–P iters/sec to rad-eq".  The
second half is the reference's T–P loop run to its own convergence test (core.py:273-338,
301-318: more than ``n_zero_crossings`` sign flips of the absorb-sweep dT in every layer, or
|dT| below ``convergence_dT``) on config C3/C4 — 60 layers × 500,000 λ × 8 species — exactly
as bench.py's ``rad_eq`` leg runs it (n_timesteps=200, n_zero_crossings=2, convergence_dT=3 K).

The oracle runs the same loop on wavelength slices in worker processes
(oracle/sharded.py: bolometric sums combined in slice order, so every slice takes the same
convergence decision).  The iteration count is integer work and must be equal; the emergent
spectrum, the F_up / F_down rows, the final T, the whole temperature history and the final
emit's dtaus are held to 1e-10 outright — no one-ulp floor is folded in (that would need a
second full oracle run; the C3 floor of one iteration is 1e-12-scale, tests/
test_gpu_fullsize_parity.py).  Both the contracted (K3) and per-species sweeps are checked
against the one oracle run.
"""
import numpy as np
import pytest

from tests.parity import assert_grid_parity, row_normwise
from oracle.sharded import ShardedOracle

pytestmark = pytest.mark.gpu

G_J, M_BAR = 2478.6519476149147, 4.0142926168559996e-24
RAD_EQ = dict(n_timesteps=200, n_zero_crossings=2, convergence_dT=3.0)


def _gpu(fa, w, tabs, precontract):
    eng = fa.Engine(w["lam"], w["p"], tabs, mmr=w["mmr"])
    try:
        eng.set_option("precontract", precontract)
        path = eng.path()
        out = eng.run(w["T0"], alpha=1.0, **RAD_EQ)
        up, down = eng.get_fluxes()
    finally:
        eng.close()
    return path, out, up, down


def test_c3_radiative_equilibrium_matches_oracle():
    import frei_amd as fa
    from frei_amd.workloads import c3
    w = c3()
    assert w["lam"].size == 500_000 and w["p"].size == 60 and len(w["names"]) == 8
    tabs = {nm: fa.SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, nm in enumerate(w["names"])}
    modes = {"contracted": -1, "per-species": 0}
    gpu = {m: _gpu(fa, w, tabs, pc) for m, pc in modes.items()}
    o_tabs = {nm: (w["base"][s], w["fp"][s], w["fT"][s], w["T_nodes"])
              for s, nm in enumerate(w["names"])}
    with ShardedOracle(o_tabs, w["lam"], w["p"], w["T0"], fa.F_TOA(w["lam"]), G_J, M_BAR,
                       mmr=w["mmr"]) as so:
        o = so.emission_spectrum(**RAD_EQ)
    sp, T, th, dt, up_o, dn_o, n_o = o
    assert 1 < n_o < RAD_EQ["n_timesteps"], f"oracle did not converge ({n_o})"
    for m, (path, out, up, down) in gpu.items():
        assert path["contracted"] == (modes[m] != 0), (m, path)
        # the integer half of the metric: the same number of T-P iterations to rad-eq
        assert out["n_iter"] == n_o, f"{m}: {out['n_iter']} iterations vs oracle {n_o}"
        assert out["temp_hist"].shape == th.shape
        assert_grid_parity(out["spectrum"], sp, up, up_o, down, dn_o,
                           f"C3 60x500000 rad-eq ({n_o} iterations) {m}",
                           T=out["final_T"], ref_T=T)
        assert float(np.max(np.abs(out["temp_hist"] - th) / th)) < 1e-10, f"{m}: T history"
        assert row_normwise(out["dtaus"], dt) < 1e-10, f"{m}: dtaus"
