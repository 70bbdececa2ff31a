"""The HIP path against the oracle at BASELINE.json's full sizes (VERDICT r02 "what's weak" #1).

- C3: 60 layers x 500,000 λ x 8 species (H2O/CO/CO2/CH4/Na/K + two CIA tables with supplied
  weights), one T-P iteration plus the final emit (core.py:273-338), contracted (K3) and
  per-species sweeps;
- C2: 60 layers x 100,000 λ, H2O + CO, T nodes = the Grid's initial temperatures (the
  reference's own table layout: n_T = n_p = 60, descending), three T-P iterations.

The oracle runs on wavelength slices in worker processes (oracle/sharded.py; the
bolometric sums are combined in slice order), with lazily built separable tables.  Criterion
(tests/parity.py assert_grid_parity): emergent spectrum elementwise and F_up / F_down
row-normwise within 1e-10, or twice the one-ulp floor of the reference algorithm on these very
inputs where that is larger (the oracle rerun with exp / expm1 one ulp high); T within 1e-10.
"""
import numpy as np
import pytest

from tests.parity import assert_grid_parity, grid_floor, row_normwise
from oracle.sharded import ShardedOracle

pytestmark = pytest.mark.gpu

G_J, M_BAR = 2478.6519476149147, 4.0142926168559996e-24
FIXED = dict(n_zero_crossings=10 ** 6, convergence_dT=-1.0)


def _gpu(fa, w, tabs, n, precontract):
    eng = fa.Engine(w["lam"], w["p"], tabs, mmr=w["mmr"])
    try:
        eng.set_option("precontract", precontract)
        path = eng.path()
        out = eng.run(w["T0"], n_timesteps=n, **FIXED)
        up, down = eng.get_fluxes()
    finally:
        eng.close()
    return path, out, up, down


def _check(fa, w, fT, n, modes):
    tabs = {nm: fa.SeparableTable(w["base"][s], w["fp"][s], fT[s], w["p"], w["T_nodes"])
            for s, nm in enumerate(w["names"])}
    gpu = {m: _gpu(fa, w, tabs, n, pc) for m, pc in modes.items()}
    o_tabs = {nm: (w["base"][s], w["fp"][s], fT[s], w["T_nodes"])
              for s, nm in enumerate(w["names"])}
    with ShardedOracle(o_tabs, w["lam"], w["p"], w["T0"], fa.F_TOA(w["lam"]), G_J, M_BAR,
                       mmr=w["mmr"]) as so:
        o = so.emission_spectrum(n_timesteps=n, **FIXED)
        pt = so.emission_spectrum(perturb=True, n_timesteps=n, **FIXED)
    floor = grid_floor(o[0], o[4], o[5], pt[0], pt[4], pt[5])
    assert o[6] == n
    for m, (path, out, up, down) in gpu.items():
        assert path["contracted"] == (modes[m] != 0), (m, path)
        assert out["n_iter"] == n
        assert np.isfinite(out["spectrum"]).all()
        what = f"{w['tag']} {w['p'].size}x{w['lam'].size} {m}"
        assert_grid_parity(out["spectrum"], o[0], up, o[4], down, o[5], what, floor,
                           T=out["final_T"], ref_T=o[1])
        assert out["temp_hist"].shape == o[2].shape
        assert float(np.max(np.abs(out["temp_hist"] - o[2]) / o[2])) < 1e-10
        assert row_normwise(out["dtaus"], o[3]) < 1e-10


def test_c3_full_size_matches_oracle():
    """C3 at full size: 1 T-P iteration + final emit, contracted and per-species."""
    import frei_amd as fa
    from frei_amd.workloads import c3
    w = c3()
    w["tag"] = "C3"
    assert w["lam"].size == 500_000 and w["p"].size == 60 and len(w["names"]) == 8
    _check(fa, w, w["fT"], 1, {"contracted": -1, "per-species": 0})


def test_c2_full_size_matches_oracle():
    """C2 at full size: 60 x 100k, H2O + CO, T nodes = the initial temperatures (n_T = n_p),
    3 T-P iterations (per-species and contracted)."""
    import frei_amd as fa
    from frei_amd.workloads import c3
    w = c3(n_lam=100_000, species=["1H2-16O", "12C-16O"])
    w["tag"] = "C2"
    w["T_nodes"] = w["T0"].copy()                    # the Grid's own nodes, descending
    fT = np.array([(w["T_nodes"] / 1000.0) ** 0.5 for _ in w["names"]])
    _check(fa, w, fT, 3, {"contracted": -1, "per-species": 0})
