"""GPU parity of the post-processing kernels (§8(f) #3) through the C ABI:
effective_temperature's per-wavelength Milne interpolation (core.py:386-405) and the
contribution function (plot.py:63-79), against the reference's own outputs on a converged
C1 atmosphere (tests/golden/post_c1.npz) and the oracle.  Tolerance: 1e-12 relative (ocml
vs libm exp/expm1/pow ulps); the Milne search index is numpy's, bit-for-bit."""
import numpy as np
import pytest

from oracle import frei_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    from frei_amd import _native as N
    assert N.device_count() >= 1, "no HIP device visible"
    return frei_amd


def _c1_grid(fa, P):
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), lam=P["lam"], pressures=P["pressures"],
                   init_temperatures=P["final_T"])
    grid.load_opacities(opacities=fa.load_example_opacity(grid, scale_factor=1))
    return grid


def test_milne_and_effective_temperature_match_reference(fa, golden):
    P = golden("post_c1.npz")
    grid = _c1_grid(fa, P)
    try:
        pm = grid.engine().milne_pressure(P["pressures"], P["dtaus"])
        assert np.all(np.abs(pm - P["p_milne"]) <= 1e-12 * np.abs(P["p_milne"]))
        spec = fa.Spectrum(P["spectrum"], P["lam"])
        tm = fa.effective_temperature_milne(grid, spec, P["dtaus"], P["final_T"])
        te = fa.effective_temperature(grid, spec, P["dtaus"], P["final_T"])
        assert abs(tm - float(P["T_milne"])) <= 1e-12 * float(P["T_milne"])
        assert abs(te - float(P["T_eff"])) <= 1e-12 * float(P["T_eff"])
    finally:
        grid._close_engine()


def test_contribution_function_matches_reference(fa, golden):
    P = golden("post_c1.npz")
    grid = _c1_grid(fa, P)
    try:
        cf = fa.contribution_function(grid, P["dtaus"], P["final_T"])
    finally:
        grid._close_engine()
    ref = P["cf_plot"]
    ok = ref != 0
    assert np.all(np.abs(cf[ok] - ref[ok]) <= 1e-12 * np.abs(ref[ok]))
    assert np.all(np.abs(cf[~ok]) <= 1e-300)


def test_post_processing_on_device_dtaus_after_run(fa):
    """After emission_spectrum the device keeps the final dtaus: T_eff and the
    contribution function use them without a host upload and match the oracle applied to
    the returned arrays (60 layers x 4096, unsorted per-layer transmissions)."""
    lam, _, _ = O.wavelength_grid(0.5, 10, 4096)
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), lam=lam, n_layers=60, T_ref=2000)
    grid.load_opacities(opacities=fa.load_example_opacity(grid, scale_factor=5))
    try:
        spec, T, th, dtaus = grid.emission_spectrum(n_timesteps=3)
        te = fa.effective_temperature(grid, spec, dtaus, T)
        ref = O.effective_temperature(lam, grid.pressures, spec.flux, dtaus, T)
        assert abs(te - ref) <= 1e-12 * ref
        pm = grid.engine().milne_pressure(grid.pressures)
        ref_pm = O.milne_pressures(dtaus, grid.pressures)
        assert np.all(np.abs(pm - ref_pm) <= 1e-12 * np.abs(ref_pm))
        cf = grid.contribution_function(T)
        ref_cf = O.contribution_function(lam, grid.pressures, T, dtaus)
        ok = ref_cf != 0
        assert np.all(np.abs(cf[ok] - ref_cf[ok]) <= 1e-12 * np.abs(ref_cf[ok]))
    finally:
        grid._close_engine()


def test_milne_search_matches_numpy_on_random_unsorted_rows(fa):
    """numpy's interp search on unsorted arrays (guess, linear-probe and bisection
    branches) for 20k random columns, including exact hits of the key."""
    rng = np.random.default_rng(3)
    nL, n = 12, 20000
    lam, _, _ = O.wavelength_grid(0.5, 10, n)
    p = np.logspace(2, -6, nL)
    dt = rng.uniform(0.0, 2.0, (nL, n))
    dt[3, ::97] = -np.log(2 / 3)              # transmission hits 2/3 (up to exp rounding)
    tabs = {"1H2-16O": fa.OpacityTable(np.ones((nL, 2, n)), p, [1000.0, 2000.0])}
    eng = fa.Engine(lam, p, tabs)
    try:
        pm = eng.milne_pressure(p, dt)
    finally:
        eng.close()
    ref = O.milne_pressures(dt, p)
    assert np.all(np.abs(pm - ref) <= 1e-12 * np.abs(ref))
