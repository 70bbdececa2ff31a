"""GPU parity: the HIP path (through the C ABI) against the reference's golden vectors
and the CPU oracle.  Criterion (tests/parity.py): |x - ref| <= 1e-10 |ref| + 4 delta cond,
cond = the oracle's first-order condition array of the reference formula."""
import numpy as np
import pytest

from oracle import frei_oracle as O
from tests.parity import (EPS, assert_flux_parity, assert_grid_parity, grid_floor,
                          perturbed_exp, rel, row_normwise)

pytestmark = pytest.mark.gpu

G_J, M_BAR = 2478.6519476149147, 4.0142926168559996e-24


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    from frei_amd import _native as N
    assert N.device_count() >= 1, "no HIP device visible"
    return frei_amd


def _cond(shape):
    return dict(up=np.zeros(shape), down=np.zeros(shape), delta=1.0)


def _floor(run, o=None):
    """One-ulp floor of an oracle run (``run()`` -> O.emission_spectrum's tuple): its outputs
    with exp / expm1 one ulp off, against the unperturbed run ``o`` (run here when None).  It is
    the spread of the reference algorithm itself, nothing else: the oracle's distance to the
    reference is checked separately (tests/test_oracle_golden.py)."""
    if o is None:
        o = run()
    with perturbed_exp():
        p = run()
    return grid_floor(o[0], o[4], o[5], p[0], p[4], p[5])


def test_propagate_fluxes_matches_reference(fa, golden):
    P = golden("propagate.npz")
    for c in range(int(P["n_cases"])):
        args = (P["lam"] * 1e-4, P[f"c{c}_F1u"], P[f"c{c}_F2d"], float(P[f"c{c}_T1"]),
                float(P[f"c{c}_T2"]), P[f"c{c}_dtau"], P[f"c{c}_omega"])
        F2u, F1d = fa.propagate_fluxes(P["lam"], P[f"c{c}_F1u"], P[f"c{c}_F2d"], args[3],
                                       args[4], P[f"c{c}_dtau"], P[f"c{c}_omega"])
        cu, cd = O.propagate_error_bound(*args, delta=1.0)
        assert_flux_parity(F2u, P[f"c{c}_F2u"], cu, what=f"case{c} F_2_up vs reference")
        assert_flux_parity(F1d, P[f"c{c}_F1d"], cd, what=f"case{c} F_1_down vs reference")
        o2u, o1d = O.propagate_fluxes(*args)
        assert_flux_parity(F2u, o2u, cu, what=f"case{c} F_2_up vs oracle")
        assert_flux_parity(F1d, o1d, cd, what=f"case{c} F_1_down vs oracle")


def test_propagate_fluxes_nonzero_g0_matches_reference(fa, golden):
    """g_0 != 0 (per-wavelength arrays of both signs and scalars) against the reference's
    own outputs; lanes where E < omega_0 are NaN in the reference and must be NaN here."""
    P = golden("propagate_g0.npz")
    for c in range(int(P["n_cases"])):
        g0 = P[f"c{c}_g0"]
        args = (P["lam"] * 1e-4, P[f"c{c}_F1u"], P[f"c{c}_F2d"], float(P[f"c{c}_T1"]),
                float(P[f"c{c}_T2"]), P[f"c{c}_dtau"], P[f"c{c}_omega"])
        F2u, F1d = fa.propagate_fluxes(P["lam"], P[f"c{c}_F1u"], P[f"c{c}_F2d"], args[3],
                                       args[4], P[f"c{c}_dtau"], P[f"c{c}_omega"], g_0=g0)
        with np.errstate(invalid="ignore"):
            cu, cd = O.propagate_error_bound(*args, delta=1.0, g_0=g0)
            o2u, o1d = O.propagate_fluxes(*args, g_0=g0)
        bad = np.isnan(P[f"c{c}_F2u"])
        assert np.array_equal(np.isnan(F2u), bad) and np.array_equal(np.isnan(F1d), bad)
        ok = ~bad
        for x, ref, cb, what in ((F2u, P[f"c{c}_F2u"], cu, "F_2_up"),
                                 (F1d, P[f"c{c}_F1d"], cd, "F_1_down"),
                                 (F2u, o2u, cu, "F_2_up vs oracle"),
                                 (F1d, o1d, cd, "F_1_down vs oracle")):
            assert_flux_parity(x[ok], ref[ok], cb[ok], what=f"g0 case{c} {what}")
    # g_0 = 0 passed explicitly is the emit/absorb form
    P0 = golden("propagate.npz")
    a = fa.propagate_fluxes(P0["lam"], P0["c0_F1u"], P0["c0_F2d"], float(P0["c0_T1"]),
                            float(P0["c0_T2"]), P0["c0_dtau"], P0["c0_omega"], g_0=0.0)
    b = fa.propagate_fluxes(P0["lam"], P0["c0_F1u"], P0["c0_F2d"], float(P0["c0_T1"]),
                            float(P0["c0_T2"]), P0["c0_dtau"], P0["c0_omega"],
                            g_0=np.zeros(P0["lam"].size))
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_kappa_matches_reference(fa, golden):
    s = golden("setup_c1.npz")
    K = golden("kappa.npz")
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), T_ref=2400)
    op = fa.load_example_opacity(grid, scale_factor=1)
    for j in range(len(K["ex_T"])):
        k, sig = fa.kappa(op, K["ex_T"][j], K["ex_p"][j], s["lam"], m_bar=M_BAR)
        assert rel(k, K["ex_k"][j]) < 1e-13, j
        assert rel(sig, K["ex_sigma"][j]) < 1e-13
    tabs2 = {n: fa.OpacityTable(O.separable_table(K[f"sep{i}_base"], K[f"sep{i}_fp"],
                                                  K[f"sep{i}_fT"]), K["sep_p"], K["sep_Tnodes"])
             for i, n in enumerate(["1H2-16O", "12C-16O"])}
    for j in range(len(K["sep_T"])):
        k, _ = fa.kappa(tabs2, K["sep_T"][j], K["sep_pq"][j], K["sep_lam"], m_bar=M_BAR)
        assert rel(k, K["sep_k"][j]) < 1e-13, j
    one = {"1H2-16O": fa.OpacityTable(
        np.clip(K["oneT_fp"][:, None, None] * K["oneT_base"][None, None, :], 1e-4, 1e3),
        K["sep_p"], [1234.0])}
    for j in range(len(K["oneT_T"])):
        k, _ = fa.kappa(one, K["oneT_T"][j], K["oneT_p"][j], K["sep_lam"], m_bar=M_BAR)
        assert rel(k, K["oneT_k"][j]) < 1e-13, j


@pytest.mark.parametrize("kind", ["emit", "absorb"])
def test_standalone_sweep_matches_reference(fa, golden, kind):
    s = golden("setup_c1.npz")
    EA = golden("emit_absorb_c1.npz")
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), T_ref=2400)
    op = fa.load_example_opacity(grid, scale_factor=1)
    fn = fa.emit if kind == "emit" else fa.absorb
    fu, fd, T, th, dtaus, dT = fn(op, grid.init_temperatures, grid.pressures, grid.lam,
                                  s["F_TOA"], G_J, m_bar=M_BAR, n_timesteps=1)
    tabs = O.example_opacity(s["pressures"], s["init_temperatures"], s["lam"], scale_factor=1)
    cond = _cond((30, 500))
    ofn = O.emit if kind == "emit" else O.absorb
    ofn(tabs, s["init_temperatures"], s["pressures"], s["lam"], s["F_TOA"], G_J, M_BAR, 1,
        err=cond)
    assert_flux_parity(fu, EA[kind + "_F_up"], cond["up"], what=kind + " F_up")
    assert_flux_parity(fd, EA[kind + "_F_down"], cond["down"], what=kind + " F_down")
    assert rel(T, EA[kind + "_T"]) < 1e-12
    assert np.max(np.abs(dT - EA[kind + "_dT"])) < 1e-8
    assert row_normwise(dtaus, EA[kind + "_dtaus"]) < 1e-13


def test_single_sweep_from_identical_state_matches_oracle(fa):
    """Strict single-sweep check (delta = eps) from a non-trivial state, 2 species."""
    rng = np.random.default_rng(3)
    lam, _, _ = O.wavelength_grid(0.5, 10, 1024)
    p = O.pressure_grid(24, -6, np.log10(200))
    T = O.temperature_grid(p, 1800.0, 0.1, 0.1) * (1 + 0.05 * rng.standard_normal(24))
    Tn = np.linspace(0.7 * T.min(), 1.3 * T.max(), 7)
    names = ["1H2-16O", "12C-16O"]
    tabs_o, tabs_f = {}, {}
    for i, n in enumerate(names):
        base = 10 ** rng.uniform(-2, 2, lam.size)
        fp, fT = (p / 1.0) ** 0.1, (Tn / 1000) ** 0.5
        v = O.separable_table(base, fp, fT)
        tabs_o[n] = O.Table(v, p, Tn)
        tabs_f[n] = fa.OpacityTable(v, p, Tn)
    up0 = 10 ** rng.uniform(8, 12, (24, lam.size))
    down0 = 10 ** rng.uniform(6, 11, (24, lam.size))
    Ft = O.F_TOA(lam)
    for kind in ("emit", "absorb"):
        cond = _cond((24, lam.size))
        ofn = O.emit if kind == "emit" else O.absorb
        ou, od, oT, odt, odT = ofn(tabs_o, T, p, lam, Ft, G_J, M_BAR, 1, up0.copy(),
                                   down0.copy(), err=cond)
        fn = fa.emit if kind == "emit" else fa.absorb
        up, down = up0.copy(), down0.copy()
        fu, fd, fT_, _, fdt, fdT = fn(tabs_f, T, p, lam, Ft, G_J, m_bar=M_BAR, n_timesteps=1,
                                      fluxes_up=up, fluxes_down=down)
        assert fu is up and fd is down            # in-place update like the reference
        assert_flux_parity(fu, ou, cond["up"], EPS, kind + " F_up")
        assert_flux_parity(fd, od, cond["down"], EPS, kind + " F_down")
        assert rel(fT_, oT) < 1e-12
        assert row_normwise(fdt, odt) < 1e-14


def test_cold_layers_planck_overflow_matches_oracle(fa):
    """Layers cold enough that hc/(lambda k T) passes 623 (expm1 >= 2^900: the sweep's
    guard-free division hands those lanes to the IEEE one) and 709.78 (expm1 = inf, B = 0),
    at short wavelengths: one sweep each way must still match the oracle strictly."""
    rng = np.random.default_rng(17)
    lam, _, _ = O.wavelength_grid(0.3, 10, 1024)
    nL = 24
    p = O.pressure_grid(nL, -6, np.log10(200))
    T = np.geomspace(1500.0, 30.0, nL)            # bottom hot, top 30 K
    x = O.H * O.C / (lam[None, :] * 1e-4 * O.K_B * T[:, None])
    assert (x > 709.8).any() and ((x > 623.0) & (x < 709.7)).any()
    Tn = np.linspace(0.9 * T.min(), 1.1 * T.max(), 9)
    v = O.separable_table(10 ** rng.uniform(-2, 2, lam.size), (p / 1.0) ** 0.1,
                          (Tn / 1000) ** 0.5)
    tabs_o = {"1H2-16O": O.Table(v, p, Tn)}
    tabs_f = {"1H2-16O": fa.OpacityTable(v, p, Tn)}
    up0 = 10 ** rng.uniform(8, 12, (nL, lam.size))
    down0 = 10 ** rng.uniform(6, 11, (nL, lam.size))
    Ft = O.F_TOA(lam)
    for kind in ("emit", "absorb"):
        cond = _cond((nL, lam.size))
        ofn = O.emit if kind == "emit" else O.absorb
        with np.errstate(over="ignore", divide="ignore", invalid="ignore"):
            ou, od, oT, odt, odT = ofn(tabs_o, T, p, lam, Ft, G_J, M_BAR, 1, up0.copy(),
                                       down0.copy(), err=cond)
        fn = fa.emit if kind == "emit" else fa.absorb
        fu, fd, fT_, _, fdt, fdT = fn(tabs_f, T, p, lam, Ft, G_J, m_bar=M_BAR, n_timesteps=1,
                                      fluxes_up=up0.copy(), fluxes_down=down0.copy())
        assert np.isfinite(fu).all() and np.isfinite(fd).all()
        assert_flux_parity(fu, ou, cond["up"], EPS, kind + " F_up (cold)")
        assert_flux_parity(fd, od, cond["down"], EPS, kind + " F_down (cold)")
        assert row_normwise(fdt, odt) < 1e-14


def test_deep_atmosphere_sweeps_match_oracle(fa):
    """400 layers: the step table no longer fits the LDS budget, so the sweep reads it from
    global memory (no LDS staging, one lane per wavelength); one sweep each way must match
    the oracle strictly."""
    rng = np.random.default_rng(23)
    lam, _, _ = O.wavelength_grid(0.5, 10, 700)
    nL = 400
    p = O.pressure_grid(nL, -6, np.log10(200))
    T = O.temperature_grid(p, 1500.0, 0.1, 0.1)
    Tn = np.linspace(0.8 * T.min(), 1.2 * T.max(), 6)
    names = ["1H2-16O", "12C-16O"]
    tabs_o, tabs_f = {}, {}
    for n in names:
        v = O.separable_table(10 ** rng.uniform(-3, 2, lam.size), (p / 1.0) ** 0.1,
                              (Tn / 1000) ** 0.5)
        tabs_o[n] = O.Table(v, p, Tn)
        tabs_f[n] = fa.OpacityTable(v, p, Tn)
    up0 = 10 ** rng.uniform(8, 12, (nL, lam.size))
    down0 = 10 ** rng.uniform(6, 11, (nL, lam.size))
    Ft = O.F_TOA(lam)
    for kind in ("emit", "absorb"):
        cond = _cond((nL, lam.size))
        ofn = O.emit if kind == "emit" else O.absorb
        ou, od, oT, odt, odT = ofn(tabs_o, T, p, lam, Ft, G_J, M_BAR, 1, up0.copy(),
                                   down0.copy(), err=cond)
        fn = fa.emit if kind == "emit" else fa.absorb
        fu, fd, fT_, _, fdt, fdT = fn(tabs_f, T, p, lam, Ft, G_J, m_bar=M_BAR, n_timesteps=1,
                                      fluxes_up=up0.copy(), fluxes_down=down0.copy())
        assert_flux_parity(fu, ou, cond["up"], EPS, kind + " F_up (deep)")
        assert_flux_parity(fd, od, cond["down"], EPS, kind + " F_down (deep)")
        # thin layers: dT = div(F_net)/... cancels between nearly equal bolometric sums, whose
        # summation order differs (fixed tree vs np.trapz), so T meets the north-star 1e-10
        assert rel(fT_, oT) < 1e-10
        assert row_normwise(fdt, odt) < 1e-14


@pytest.mark.parametrize("n_lam,nL,S", [(3, 4, 1), (63, 5, 2), (65, 7, 1), (129, 33, 3),
                                         (257, 6, 2), (1000, 9, 1)])
def test_ragged_shapes_sweeps_match_oracle(fa, n_lam, nL, S):
    """Edge shapes: wavelength counts around the 64/128/256-lane block sizes of the one-lane
    and grouped-lane sweeps, the fewest layers, odd step counts; one sweep each way."""
    rng = np.random.default_rng(1000 * n_lam + nL)
    lam, _, _ = O.wavelength_grid(0.5, 10, n_lam)
    p = O.pressure_grid(nL, -6, np.log10(200))
    T = O.temperature_grid(p, 1700.0, 0.1, 0.1) * (1 + 0.03 * rng.standard_normal(nL))
    Tn = np.linspace(0.7 * T.min(), 1.3 * T.max(), 5)
    names = ["1H2-16O", "12C-16O", "Na"][:S]
    tabs_o, tabs_f = {}, {}
    for n in names:
        v = O.separable_table(10 ** rng.uniform(-3, 2, lam.size), (p / 1.0) ** 0.1,
                              (Tn / 1000) ** 0.5)
        tabs_o[n] = O.Table(v, p, Tn)
        tabs_f[n] = fa.OpacityTable(v, p, Tn)
    up0 = 10 ** rng.uniform(8, 12, (nL, lam.size))
    down0 = 10 ** rng.uniform(6, 11, (nL, lam.size))
    Ft = O.F_TOA(lam)
    for kind in ("emit", "absorb"):
        cond = _cond((nL, lam.size))
        ofn = O.emit if kind == "emit" else O.absorb
        ou, od, oT, odt, odT = ofn(tabs_o, T, p, lam, Ft, G_J, M_BAR, 1, up0.copy(),
                                   down0.copy(), err=cond)
        fn = fa.emit if kind == "emit" else fa.absorb
        fu, fd, fT_, _, fdt, fdT = fn(tabs_f, T, p, lam, Ft, G_J, m_bar=M_BAR, n_timesteps=1,
                                      fluxes_up=up0.copy(), fluxes_down=down0.copy())
        assert_flux_parity(fu, ou, cond["up"], EPS, f"{kind} F_up {n_lam}x{nL}")
        assert_flux_parity(fd, od, cond["down"], EPS, f"{kind} F_down {n_lam}x{nL}")
        assert rel(fT_, oT) < 1e-10
        assert row_normwise(fdt, odt) < 1e-14


def _grid_run(fa, C, pre, tabs_f, tabs_o, lam, p, T0, n, Ft=None):
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), lam=lam, pressures=p, init_temperatures=T0)
    grid.load_opacities(opacities=tabs_f)
    spec, T, th, dtaus = grid.emission_spectrum(n_timesteps=n)
    cond = _cond((len(p), len(lam)))
    Ft = O.F_TOA(lam) if Ft is None else Ft
    o = O.emission_spectrum(tabs_o, T0, p, lam, Ft, G_J, M_BAR, 1, n_timesteps=n, err=cond)
    relT = rel(T, C[pre + "final_T"])
    assert relT < 1e-10, relT
    delta = max(EPS, relT)
    assert_flux_parity(spec.flux, C[pre + "spectrum"], cond["up"][-1], delta, pre + "spectrum")
    assert rel(th, C[pre + "temp_hist"]) < 1e-10
    assert th.shape == C[pre + "temp_hist"].shape
    assert row_normwise(dtaus, C[pre + "dtaus"]) < 1e-10
    up, down = grid.engine().get_fluxes()
    assert_flux_parity(up, C[pre + "F_up"], cond["up"], delta, pre + "F_up")
    assert_flux_parity(down, C[pre + "F_down"], cond["down"], delta, pre + "F_down")
    floor = _floor(lambda: O.emission_spectrum(tabs_o, T0, p, lam, Ft, G_J, M_BAR, 1,
                                               n_timesteps=n), o)
    # the GPU against the oracle on the same inputs (tolerance: 1e-10 or 2x the one-ulp floor)
    assert_grid_parity(spec.flux, o[0], up, o[4], down, o[5], pre + " vs oracle", floor,
                       T=T, ref_T=o[1])
    # and against the reference's own outputs (the same floor; the oracle's own distance to
    # them is pinned separately, tests/test_oracle_golden.py)
    assert_grid_parity(spec.flux, C[pre + "spectrum"], up, C[pre + "F_up"], down,
                       C[pre + "F_down"], pre + " vs reference", floor, T=T,
                       ref_T=C[pre + "final_T"])
    return grid, spec, T, dtaus


def test_c1_emission_spectrum_matches_reference(fa, golden):
    s = golden("setup_c1.npz")
    C = golden("c1_step1.npz")
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), T_ref=2400)
    tabs_f = fa.load_example_opacity(grid, scale_factor=1)
    tabs_o = O.example_opacity(s["pressures"], s["init_temperatures"], s["lam"], scale_factor=1)
    g, spec, T, dtaus = _grid_run(fa, C, "ex_", tabs_f, tabs_o, s["lam"], s["pressures"],
                                  s["init_temperatures"], 1)
    assert rel(spec.flux, C["ex_spectrum"]) < 1e-10    # emergent spectrum, elementwise
    teff = fa.effective_temperature(g, spec, dtaus, T)
    assert abs(teff - float(C["ex_Teff"])) < 1e-6
    gray_o = {"1H2-16O": O.Table(np.ones((30, 30, 500)), s["pressures"], s["init_temperatures"])}
    gray_f = {"1H2-16O": fa.OpacityTable(np.ones((30, 30, 500)), s["pressures"],
                                         s["init_temperatures"])}
    _grid_run(fa, C, "gray_", gray_f, gray_o, s["lam"], s["pressures"], s["init_temperatures"], 1)


def test_c1_converges_in_50_iterations_like_reference(fa, golden):
    s = golden("setup_c1.npz")
    C = golden("c1_converge.npz")
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), T_ref=2400)
    tabs_f = fa.load_example_opacity(grid, scale_factor=1)
    tabs_o = O.example_opacity(s["pressures"], s["init_temperatures"], s["lam"], scale_factor=1)
    _, spec, T, _ = _grid_run(fa, C, "cv_", tabs_f, tabs_o, s["lam"], s["pressures"],
                              s["init_temperatures"], 100)
    assert rel(spec.flux, C["cv_spectrum"]) < 1e-10


def test_c2small_two_species_matches_reference(fa, golden):
    C = golden("c2small.npz")
    names = ["1H2-16O", "12C-16O"]
    tabs_o = {n: O.Table(O.separable_table(C[f"s{i}_base"], C[f"s{i}_fp"], C[f"s{i}_fT"]),
                         C["pressures"], C["T_nodes"]) for i, n in enumerate(names)}
    tabs_f = {n: fa.SeparableTable(C[f"s{i}_base"], C[f"s{i}_fp"], C[f"s{i}_fT"],
                                   C["pressures"], C["T_nodes"]) for i, n in enumerate(names)}
    _grid_run(fa, C, "", tabs_f, tabs_o, C["lam"], C["pressures"], C["init_temperatures"], 3)


def test_c2strong_two_species_matches_reference_outright(fa, golden):
    """c2small's well-conditioned twin, made by the reference itself (make_goldens.py
    case_c2strong: the same 60 x 2048 grid and line forests at 1e3x strength, clipped to
    [10, 1e3] cm^2 g^-1; the reference's own one-ulp floor 3e-13): three T-P iterations on the
    GPU against the reference's outputs and against the oracle at 1e-10 outright — no floor
    rule."""
    C = golden("c2strong.npz")
    lo, hi = float(C["clip_lo"]), float(C["clip_hi"])
    names = ["1H2-16O", "12C-16O"]
    tabs_o = {n: O.Table(O.separable_table(C[f"s{i}_base"], C[f"s{i}_fp"], C[f"s{i}_fT"], lo, hi),
                         C["pressures"], C["T_nodes"]) for i, n in enumerate(names)}
    tabs_f = {n: fa.SeparableTable(C[f"s{i}_base"], C[f"s{i}_fp"], C[f"s{i}_fT"], C["pressures"],
                                   C["T_nodes"], lo=lo, hi=hi) for i, n in enumerate(names)}
    lam, p, T0 = C["lam"], C["pressures"], C["init_temperatures"]
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), lam=lam, pressures=p, init_temperatures=T0)
    grid.load_opacities(opacities=tabs_f)
    spec, T, th, dtaus = grid.emission_spectrum(n_timesteps=3)
    up, down = grid.engine().get_fluxes()
    o = O.emission_spectrum(tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1, n_timesteps=3)
    for ref, what in (((C["spectrum"], C["F_up"], C["F_down"], C["final_T"]), "vs reference"),
                      ((o[0], o[4], o[5], o[1]), "vs oracle")):
        e = assert_grid_parity(spec.flux, ref[0], up, ref[1], down, ref[2],
                               f"c2strong {what} (outright)", T=T, ref_T=ref[3])
        assert e["within_1e-10"], e
    assert rel(th, C["temp_hist"]) < 1e-10 and th.shape == C["temp_hist"].shape
    assert row_normwise(dtaus, C["dtaus"]) < 1e-10


def test_eight_species_device_tables_match_oracle(fa):
    """C3-like: 8 species (6 molecules + 2 CIA-style tables with supplied weights),
    device-generated separable tables, 60 layers x 4096, two T-P iterations."""
    rng = np.random.default_rng(11)
    lam, _, _ = O.wavelength_grid(0.5, 10, 4096)
    p = O.pressure_grid(60, -6, np.log10(200))
    T0 = O.temperature_grid(p, 1500.0, 0.1, 0.1)
    Tn = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 16)
    names = ["1H2-16O", "12C-16O", "12C-16O2", "12C-1H4", "Na", "K", "H2-H2", "H2-He"]
    mmr = np.vstack([O.mock_mmr(names[:6], M_BAR)[:, None] * np.ones(60),
                     1e-3 * (p / p[0]) ** 0.5, 5e-4 * np.ones(60)])
    tabs_o, tabs_f = {}, {}
    for i, n in enumerate(names):
        base = 10 ** (rng.uniform(-3, 1, lam.size))
        fp, fT = (p / 1.0) ** 0.1, (Tn / 1000.0) ** 0.5
        tabs_o[n] = O.Table(O.separable_table(base, fp, fT), p, Tn)
        tabs_f[n] = fa.SeparableTable(base, fp, fT, p, Tn)
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), lam=lam, pressures=p, init_temperatures=T0)
    grid.load_opacities(opacities=tabs_f, mmr=mmr)
    spec, T, th, dtaus = grid.emission_spectrum(n_timesteps=2, n_zero_crossings=10**6,
                                                convergence_dT=-1)
    cond = _cond((60, lam.size))
    osp, oT, oth, odt, ou, od, it = O.emission_spectrum(
        tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1, n_timesteps=2,
        n_zero_crossings=10**6, convergence_dT=-1, mmr=mmr, err=cond)
    relT = rel(T, oT)
    assert relT < 1e-10
    assert th.shape == (60, 4)
    delta = max(EPS, relT)
    assert_flux_parity(spec.flux, osp, cond["up"][-1], delta, "spectrum")
    up, down = grid.engine().get_fluxes()
    assert_flux_parity(up, ou, cond["up"], delta, "F_up")
    assert_flux_parity(down, od, cond["down"], delta, "F_down")
    floor = _floor(lambda: O.emission_spectrum(
        tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1, n_timesteps=2,
        n_zero_crossings=10**6, convergence_dT=-1, mmr=mmr))
    assert_grid_parity(spec.flux, osp, up, ou, down, od, "8 species", floor, T=T, ref_T=oT)
    assert row_normwise(dtaus, odt) < 1e-10


def test_nan_in_table_is_skipped_like_xarray_sum(fa):
    """Q8: for S > 1 the species sum skips NaN (xarray nansum); the device NaN scan must
    switch the sweep to its NaN-checking variant."""
    rng = np.random.default_rng(21)
    lam, _, _ = O.wavelength_grid(0.5, 10, 640)
    p = O.pressure_grid(16, -6, np.log10(200))
    T0 = O.temperature_grid(p, 1800.0, 0.1, 0.1)
    Tn = np.linspace(0.7 * T0.min(), 1.3 * T0.max(), 6)
    names = ["1H2-16O", "12C-16O"]
    vals = [O.separable_table(10 ** rng.uniform(-2, 1, lam.size), (p / 1.0) ** 0.1,
                              (Tn / 1000) ** 0.5) for _ in names]
    vals[1] = vals[1].copy()
    vals[1][:, :, 100:140] = np.nan     # a NaN band in the second species
    tabs_o = {n: O.Table(v, p, Tn) for n, v in zip(names, vals)}
    tabs_f = {n: fa.OpacityTable(v, p, Tn) for n, v in zip(names, vals)}
    k, _ = fa.kappa(tabs_f, T0[3], p[3], lam, m_bar=M_BAR)
    ko, _ = O.kappa(tabs_o, T0[3], p[3], lam, M_BAR)
    assert np.all(np.isfinite(k)) and rel(k, ko) < 1e-14
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), lam=lam, pressures=p, init_temperatures=T0)
    grid.load_opacities(opacities=tabs_f)
    spec, T, th, dtaus = grid.emission_spectrum(n_timesteps=2)
    cond = _cond((16, lam.size))
    osp, oT, oth, odt, ou, od, it = O.emission_spectrum(tabs_o, T0, p, lam, O.F_TOA(lam), G_J,
                                                        M_BAR, 1, n_timesteps=2, err=cond)
    relT = rel(T, oT)
    assert relT < 1e-10 and np.all(np.isfinite(spec.flux))
    assert_flux_parity(spec.flux, osp, cond["up"][-1], max(EPS, relT), "spectrum with NaN band")
    up, down = grid.engine().get_fluxes()
    floor = _floor(lambda: O.emission_spectrum(tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1,
                                               n_timesteps=2))
    assert_grid_parity(spec.flux, osp, up, ou, down, od, "NaN band", floor, T=T, ref_T=oT)


@pytest.mark.parametrize("mode", ["single_T", "offnode_p", "mixed_T"])
def test_generic_sweep_path_matches_oracle(fa, mode):
    """Tables the fast kernel cannot take run the generic sweep kernel: a single-temperature
    table (pressure-only interp1d, opacity.py:256-259) or table pressure nodes that are not
    the grid's (full bilinear interpolation, 4 corners). "mixed_T": species with different
    temperature nodes run the fast kernel with one bracket per species (no shared bracket)."""
    rng = np.random.default_rng(31)
    lam, _, _ = O.wavelength_grid(0.5, 10, 900)
    p = O.pressure_grid(18, -6, np.log10(200))
    T0 = O.temperature_grid(p, 2000.0, 0.1, 0.1)
    names = ["1H2-16O", "12C-16O"]
    if mode == "single_T":
        pn, Tns = p, [np.array([1500.0])] * 2
    elif mode == "offnode_p":
        pn = np.logspace(np.log10(300), -7, 11)        # coarser, not on the layer grid
        Tns = [np.linspace(0.7 * T0.min(), 1.3 * T0.max(), 5)] * 2
    else:
        pn = p
        Tns = [np.linspace(0.7 * T0.min(), 1.3 * T0.max(), 5),
               np.linspace(0.6 * T0.min(), 1.4 * T0.max(), 7)]
    vals = [O.separable_table(10 ** rng.uniform(-2, 1, lam.size), (pn / 1.0) ** 0.1,
                              (Tn / 1000) ** 0.5) for Tn in Tns]
    tabs_o = {n: O.Table(v, pn, Tn) for n, v, Tn in zip(names, vals, Tns)}
    tabs_f = {n: fa.OpacityTable(v, pn, Tn) for n, v, Tn in zip(names, vals, Tns)}
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), lam=lam, pressures=p, init_temperatures=T0)
    grid.load_opacities(opacities=tabs_f)
    spec, T, th, dtaus = grid.emission_spectrum(n_timesteps=3)
    cond = _cond((18, lam.size))
    osp, oT, oth, odt, ou, od, it = O.emission_spectrum(tabs_o, T0, p, lam, O.F_TOA(lam), G_J,
                                                        M_BAR, 1, n_timesteps=3, err=cond)
    relT = rel(T, oT)
    assert relT < 1e-10, relT
    delta = max(EPS, relT)
    assert_flux_parity(spec.flux, osp, cond["up"][-1], delta, mode + " spectrum")
    up, down = grid.engine().get_fluxes()
    assert_flux_parity(up, ou, cond["up"], delta, mode + " F_up")
    assert_flux_parity(down, od, cond["down"], delta, mode + " F_down")
    floor = _floor(lambda: O.emission_spectrum(tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1,
                                               n_timesteps=3))
    assert_grid_parity(spec.flux, osp, up, ou, down, od, mode, floor, T=T, ref_T=oT)
    assert row_normwise(dtaus, odt) < 1e-10


def test_species_contraction_matches_per_species_sum(fa, monkeypatch):
    """K3: the precontracted table (sum_s mmr_s tab_s per node row, then interpolation)
    against the in-sweep per-species sum (FREI_PRECONTRACT=0) and the oracle, 8 species
    with layer-dependent mmr, 3 T-P iterations."""
    rng = np.random.default_rng(5)
    lam, _, _ = O.wavelength_grid(0.5, 10, 3000)
    p = O.pressure_grid(40, -6, np.log10(200))
    T0 = O.temperature_grid(p, 1700.0, 0.1, 0.1)
    Tn = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 12)
    names = ["1H2-16O", "12C-16O", "12C-16O2", "12C-1H4", "Na", "K", "H2-H2", "H2-He"]
    mmr = np.vstack([O.mock_mmr(names[:6], M_BAR)[:, None] * np.ones(40),
                     1e-3 * (p / p[0]) ** 0.5, 5e-4 * np.ones(40)])
    tabs_o, tabs_f = {}, {}
    for n in names:
        base = 10 ** rng.uniform(-3, 1, lam.size)
        fp, fT = (p / 1.0) ** 0.1, (Tn / 1000.0) ** 0.5
        tabs_o[n] = O.Table(O.separable_table(base, fp, fT), p, Tn)
        tabs_f[n] = fa.SeparableTable(base, fp, fT, p, Tn)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("FREI_PRECONTRACT", mode)
        eng = fa.Engine(lam, p, tabs_f, mmr=mmr)
        try:
            assert eng.path()["contracted"] == (mode == "1")
            out[mode] = eng.run(T0, n_timesteps=3, n_zero_crossings=10 ** 6,
                                convergence_dT=-1.0)
            out[mode]["fluxes"] = eng.get_fluxes()
        finally:
            eng.close()
    cond = _cond((40, lam.size))
    osp, oT, oth, odt, ou, od, it = O.emission_spectrum(
        tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1, n_timesteps=3,
        n_zero_crossings=10 ** 6, convergence_dT=-1, mmr=mmr, err=cond)
    floor = _floor(lambda: O.emission_spectrum(
        tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1, n_timesteps=3,
        n_zero_crossings=10 ** 6, convergence_dT=-1, mmr=mmr))
    for mode in ("1", "0"):
        relT = rel(out[mode]["final_T"], oT)
        assert relT < 1e-10
        delta = max(EPS, relT)
        assert_flux_parity(out[mode]["spectrum"], osp, cond["up"][-1], delta, "spectrum " + mode)
        up, down = out[mode]["fluxes"]
        assert_flux_parity(up, ou, cond["up"], delta, "F_up " + mode)
        assert_flux_parity(down, od, cond["down"], delta, "F_down " + mode)
        assert_grid_parity(out[mode]["spectrum"], osp, up, ou, down, od,
                           "contracted" if mode == "1" else "per-species", floor,
                           T=out[mode]["final_T"], ref_T=oT)


@pytest.mark.parametrize("waves", [4, 8])          # waves per block (8: two per SIMD, lockstep)
@pytest.mark.parametrize("red_mode", ["stage", "rows", "full"])   # partial-sum layouts
@pytest.mark.parametrize("n_layers", [34, 36])     # 33 / 35 steps: dummy group slots
def test_grouped_lane_sweep_matches_one_lane_form(fa, monkeypatch, n_layers, red_mode, waves):
    """The grouped-lane sweeps (two or four lanes per wavelength, small slices; 4- or 8-wave
    blocks) form every flux with the one-lane expressions: one sweep from the same state gives
    bit-identical fluxes and dtaus; only the bolometric partial sums use another fixed summation
    tree (dT within 1e-10), so T-P iterations agree within the parity tolerance."""
    rng = np.random.default_rng(9)
    lam, _, _ = O.wavelength_grid(0.5, 10, 5000)
    p = O.pressure_grid(n_layers, -6, np.log10(200))
    T0 = O.temperature_grid(p, 1600.0, 0.1, 0.1)
    Tn = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 9)
    names = ["1H2-16O", "12C-16O", "Na"]
    tabs = {n: fa.SeparableTable(10 ** rng.uniform(-4, 2, lam.size), (p / 1.0) ** 0.1,
                                 (Tn / 1000.0) ** 0.5, p, Tn) for n in names}
    mmr = O.mock_mmr(names, M_BAR)[:, None] * np.ones(n_layers)
    out = {}
    monkeypatch.setenv("FREI_RED_STAGE", "1" if red_mode == "stage" else "0")
    monkeypatch.setenv("FREI_RED_ROWS", "1" if red_mode == "rows" else "0")
    monkeypatch.setenv("FREI_GROUP_WAVES", str(waves))
    for q in (4, 2, 1):
        monkeypatch.setenv("FREI_GROUP_Q", str(q))
        eng = fa.Engine(lam, p, tabs, mmr=mmr)
        try:
            path = eng.path()
            assert (path["paired"], path["quad"]) == (q == 2, q == 4)
            r = {}
            for d in (0, 1):    # emit then absorb from the same initial state
                eng.set_temperatures(T0)
                eng.set_fluxes(np.full((n_layers, lam.size), 1e9),
                               np.full((n_layers, lam.size), 2e8))
                r[d] = eng.sweep(d, alpha=1.0) + eng.get_fluxes()
            r["run"] = eng.run(T0, n_timesteps=4, n_zero_crossings=10 ** 6,
                               convergence_dT=-1.0)
            out[q] = r
        finally:
            eng.close()
    for q in (4, 2):
        for d in (0, 1):
            dT_p, bol_p, dt_p, up_p, dn_p = out[q][d]
            dT_o, bol_o, dt_o, up_o, dn_o = out[1][d]
            assert np.array_equal(up_p, up_o) and np.array_equal(dn_p, dn_o), f"Q{q} dir {d}"
            assert np.array_equal(dt_p, dt_o), f"Q{q} dir {d} dtaus"
            assert row_normwise(bol_p, bol_o) < 1e-12
            assert np.all(np.abs(dT_p - dT_o) <= 1e-10 * np.abs(dT_o) + 1e-300)
        assert rel(out[q]["run"]["final_T"], out[1]["run"]["final_T"]) < 1e-12
        assert row_normwise(out[q]["run"]["spectrum"], out[1]["run"]["spectrum"]) < 1e-9


# 4 steps (one partial phase) / 33 / 36 / 59 / 79 steps: partial phases; 80 layers needs more
# LDS than the earlier cases (the kernel's dynamic-LDS opt-in is raised between launches)
@pytest.mark.parametrize("n_layers", [5, 34, 37, 60, 80])
def test_pipe_sweep_matches_one_lane_form(fa, monkeypatch, n_layers):
    """The producer/consumer sweep (three producer waves form the step coefficients into an LDS
    ring, one consumer wave runs the carried chain) uses the one-lane expressions in the same
    order: fluxes and dtaus are bit-identical for 1, 2 and 4 consumers per block; with 4 (256
    wavelengths per block, the one-lane block) the bolometric partials are too, so a T-P run
    gives bit-identical temperatures and spectra; with 1 or 2 only the block-sum tree differs."""
    rng = np.random.default_rng(17)
    lam, _, _ = O.wavelength_grid(0.5, 10, 5000)   # 5000: a ragged last block for every form
    p = O.pressure_grid(n_layers, -6, np.log10(200))
    T0 = O.temperature_grid(p, 1600.0, 0.1, 0.1)
    Tn = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 9)
    names = ["1H2-16O", "12C-16O", "Na"]
    tabs = {n: fa.SeparableTable(10 ** rng.uniform(-4, 2, lam.size), (p / 1.0) ** 0.1,
                                 (Tn / 1000.0) ** 0.5, p, Tn) for n in names}
    mmr = O.mock_mmr(names, M_BAR)[:, None] * np.ones(n_layers)
    monkeypatch.setenv("FREI_GROUP_Q", "1")
    out = {}
    for nc in (0, 1, 2, 4):
        monkeypatch.setenv("FREI_PIPE", str(nc))
        eng = fa.Engine(lam, p, tabs, mmr=mmr)
        try:
            path = eng.path()
            assert path["contracted"] and path["pipe"] == nc, path
            r = {}
            for d in (0, 1):    # emit then absorb from the same initial state
                eng.set_temperatures(T0)
                eng.set_fluxes(np.full((n_layers, lam.size), 1e9),
                               np.full((n_layers, lam.size), 2e8))
                r[d] = eng.sweep(d, alpha=1.0) + eng.get_fluxes()
            r["run"] = eng.run(T0, n_timesteps=4, n_zero_crossings=10 ** 6,
                               convergence_dT=-1.0)
            r["fl"] = eng.get_fluxes()
            out[nc] = r
        finally:
            eng.close()
    for nc in (1, 2, 4):
        for d in (0, 1):
            dT_p, bol_p, dt_p, up_p, dn_p = out[nc][d]
            dT_o, bol_o, dt_o, up_o, dn_o = out[0][d]
            assert np.array_equal(up_p, up_o) and np.array_equal(dn_p, dn_o), f"NC{nc} dir {d}"
            assert np.array_equal(dt_p, dt_o), f"NC{nc} dir {d} dtaus"
            if nc == 4:
                assert np.array_equal(bol_p, bol_o) and np.array_equal(dT_p, dT_o)
            else:
                assert row_normwise(bol_p, bol_o) < 1e-12
                assert np.all(np.abs(dT_p - dT_o) <= 1e-10 * np.abs(dT_o) + 1e-300)
        ro, rp = out[0]["run"], out[nc]["run"]
        if nc == 4:
            assert np.array_equal(rp["final_T"], ro["final_T"])
            assert np.array_equal(rp["spectrum"], ro["spectrum"])
            assert all(np.array_equal(a, b) for a, b in zip(out[nc]["fl"], out[0]["fl"]))
            assert np.array_equal(rp["dtaus"], ro["dtaus"])
        else:
            assert rel(rp["final_T"], ro["final_T"]) < 1e-12
            assert row_normwise(rp["spectrum"], ro["spectrum"]) < 1e-9


@pytest.mark.parametrize("form", [("1", "0"), ("2", "0"), ("4", "0"), ("1", "4"), ("1", "1")])
def test_step_records_formed_in_sweep_are_bitwise_the_updates(fa, monkeypatch, form):
    """With shared brackets on the contracted table the sweeps form their own step records from
    the current temperatures (FREI_REC_SWEEP; by default in every form but the producer/consumer
    sweep, forced here for all) and the update kernel writes none: a
    T-P run gives bitwise the temperatures, spectrum, fluxes and dtaus of the update-written
    records, in every sweep form (one-lane with LDS records, two / four lanes per wavelength,
    producer/consumer with 4 and 1 consumers)."""
    q, nc = form
    rng = np.random.default_rng(5)
    lam, _, _ = O.wavelength_grid(0.5, 10, 3000)
    nL = 33
    p = O.pressure_grid(nL, -6, np.log10(200))
    T0 = O.temperature_grid(p, 1600.0, 0.1, 0.1)
    Tn = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 9)
    names = ["1H2-16O", "12C-16O"]
    tabs = {n: fa.SeparableTable(10 ** rng.uniform(-4, 2, lam.size), (p / 1.0) ** 0.1,
                                 (Tn / 1000.0) ** 0.5, p, Tn) for n in names}
    mmr = O.mock_mmr(names, M_BAR)[:, None] * np.ones(nL)
    monkeypatch.setenv("FREI_GROUP_Q", q)
    monkeypatch.setenv("FREI_PIPE", nc)
    out = {}
    for rec in ("0", "1"):
        monkeypatch.setenv("FREI_REC_SWEEP", rec)   # 1: every form (the default skips the pipe)
        eng = fa.Engine(lam, p, tabs, mmr=mmr)
        try:
            path = eng.path()
            assert path["contracted"] and path["lds_steps"] and path["pipe"] == int(nc)
            r = eng.run(T0, n_timesteps=5, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            out[rec] = (r, eng.get_fluxes())
        finally:
            eng.close()
    (a, fa_), (b, fb_) = out["0"], out["1"]
    for k in ("final_T", "spectrum", "dtaus", "temp_hist"):
        assert np.array_equal(a[k], b[k]), k
    assert all(np.array_equal(x, y) for x, y in zip(fa_, fb_))


def test_shims_reuse_device_context_and_vector_kappa(fa, golden):
    """emit/absorb/kappa keep their device context (uploaded tables) between calls with the
    same opacity dict: repeated calls hit the cache and give bitwise-identical results; kappa
    also takes arrays of (T, p) points along one dimension (opacity.py:235-263)."""
    from frei_amd import engine as E
    E.clear_engine_cache()
    s = golden("setup_c1.npz")
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), T_ref=2400)
    op = fa.load_example_opacity(grid, scale_factor=1)
    args = (op, grid.init_temperatures, grid.pressures, grid.lam, s["F_TOA"], G_J)
    r1 = fa.emit(*args, m_bar=M_BAR, n_timesteps=1)
    assert len(E._ENGINE_CACHE) == 1
    eng = E._ENGINE_CACHE[0][2]
    r2 = fa.emit(*args, m_bar=M_BAR, n_timesteps=1)
    r3 = fa.absorb(*args, m_bar=M_BAR, n_timesteps=1)
    assert len(E._ENGINE_CACHE) == 1 and E._ENGINE_CACHE[0][2] is eng
    for x, y in zip(r1, r2):
        assert np.array_equal(x, y)
    EA = golden("emit_absorb_c1.npz")
    assert rel(r3[2], EA["absorb_T"]) < 1e-12
    K = golden("kappa.npz")
    ks = [fa.kappa(op, K["ex_T"][j], K["ex_p"][j], s["lam"], m_bar=M_BAR)[0]
          for j in range(len(K["ex_T"]))]
    assert len(E._ENGINE_CACHE) == 2                  # one kappa context for all points
    kv, sig = fa.kappa(op, K["ex_T"], K["ex_p"], s["lam"], m_bar=M_BAR)
    assert kv.shape == (len(K["ex_T"]), s["lam"].size)
    for j in range(len(K["ex_T"])):
        assert np.array_equal(kv[j], ks[j])
        assert rel(kv[j], K["ex_k"][j]) < 1e-13
    k1, _ = fa.kappa(op, K["ex_T"][:1], K["ex_p"][:1], s["lam"], m_bar=M_BAR)
    assert k1.shape == (s["lam"].size,)               # one point: flat, like the reference
    E.clear_engine_cache()
    assert not E._ENGINE_CACHE and eng._ctx is None


def _chem_table(names, T_lo=300.0, T_hi=4000.0, n_T=14, n_p=9):
    """Synthetic equilibrium-like chemistry: H2O falls and CO rises with T (log-space tanh
    around 1500 K), weak pressure dependence; mass mixing ratios on (T, log p) nodes."""
    T = np.linspace(T_lo, T_hi, n_T)
    p = np.logspace(-7, 3, n_p)
    x = np.tanh((T[:, None] - 1500.0) / 400.0) + 0.05 * np.log10(p)[None, :]
    base = O.mock_mmr(names, M_BAR)
    vals = []
    for s, n in enumerate(names):
        sign = -1.0 if s % 2 == 0 else 1.0
        vals.append(base[s] * 10 ** (0.8 * sign * x))
    return np.array(vals), T, p


@pytest.mark.parametrize("case", ["c1", "c1_strong", "c2_like"])
def test_temperature_dependent_chemistry_matches_oracle(fa, case):
    """A chemistry table (mmr on (T, p) nodes, re-interpolated at every layer's current T each
    sweep, like the reference's chemistry(T, p) call inside kappa, opacity.py:246-248): the
    sweep keeps the per-species sum (no K3), and the T-P loop matches the oracle given the same
    table (parity against FastChem itself is unpinned: it is third-party).  c1_strong: the c1
    run with opacities 10-1000 cm^2/g, whose one-ulp floor is below 1e-10 — held to 1e-10
    outright."""
    rng = np.random.default_rng(41)
    if case in ("c1", "c1_strong"):
        lam, _, _ = O.wavelength_grid(0.5, 10, 500)
        p = O.pressure_grid(30, -6, np.log10(200))
        T0 = O.temperature_grid(p, 2400.0, 0.1, 0.1)
        n_it, nzc, thr = 60, 2, 3.0
    else:
        lam, _, _ = O.wavelength_grid(0.5, 10, 2048)
        p = O.pressure_grid(60, -6, np.log10(200))
        T0 = O.temperature_grid(p, 1500.0, 0.1, 0.1)
        n_it, nzc, thr = 3, 10 ** 6, -1.0
    names = ["1H2-16O", "12C-16O", "12C-1H4"]
    Tn = np.linspace(0.7 * T0.min(), 1.3 * T0.max(), 10)
    tabs_o, tabs_f = {}, {}
    for n in names:
        base = 10 ** (rng.uniform(1, 3, lam.size) if case == "c1_strong"
                      else rng.uniform(-3, 1, lam.size))
        fp, fT = (p / 1.0) ** 0.1, (Tn / 1000.0) ** 0.5
        tabs_o[n] = O.Table(O.separable_table(base, fp, fT), p, Tn)
        tabs_f[n] = fa.SeparableTable(base, fp, fT, p, Tn)
    vals, cT, cp = _chem_table(names)
    chem_f = fa.ChemistryTable({n: vals[s] for s, n in enumerate(names)}, cT, cp)
    chem_o = O.ChemistryTable(vals, cT, cp)
    eng = fa.Engine(lam, p, tabs_f, mmr=chem_f)
    try:
        assert not eng.path()["contracted"]
        out = eng.run(T0, n_timesteps=n_it, n_zero_crossings=nzc, convergence_dT=thr)
        up, down = eng.get_fluxes()
        # kappa at arbitrary (T, p): mmr from the table at that point
        for Tq, pq in ((T0[3] * 1.1, p[3]), (T0[-5], np.sqrt(p[7] * p[8]))):
            k, _ = eng.kappa(Tq, pq)
            ko, _ = O.kappa(tabs_o, Tq, pq, lam, M_BAR, mmr=chem_o(Tq, pq))
            assert rel(k, ko) < 1e-13
    finally:
        eng.close()

    def run():
        return O.emission_spectrum(tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1,
                                   n_timesteps=n_it, n_zero_crossings=nzc, convergence_dT=thr,
                                   mmr=chem_o)
    osp, oT, oth, odt, ou, od, it = run()
    assert out["n_iter"] == it
    with perturbed_exp():
        psp, pT, _, _, pu, pd, _ = run()
    floor = grid_floor(osp, ou, od, psp, pu, pd)
    if case == "c1_strong":   # well conditioned: 1e-10 outright, no floor
        assert max(floor) <= 1e-10 and rel(pT, oT) <= 1e-10, floor
        assert rel(out["final_T"], oT) <= 1e-10
        assert_grid_parity(out["spectrum"], osp, up, ou, down, od, "chemistry " + case,
                           T=out["final_T"], ref_T=oT)
    else:
        assert rel(out["final_T"], oT) <= max(1e-10, 2 * rel(pT, oT))
        assert_grid_parity(out["spectrum"], osp, up, ou, down, od, "chemistry " + case, floor)
    # the chemistry really moved with T: mmr at the final vs the initial profile
    m0 = np.array([chem_o(t, pb) for t, pb in zip(T0, p)])
    m1 = np.array([chem_o(t, pb) for t, pb in zip(out["final_T"], p)])
    assert np.max(np.abs(m1 - m0) / m0) > 1e-3


@pytest.mark.parametrize("precontract,ptop", [("1", -6), ("0", -6), ("1", -2)])
def test_high_albedo_lanes_match_oracle(fa, monkeypatch, precontract, ptop):
    """Q9: omega_0 > 0.1 takes E(omega_0) (twostream.py:70-94) and the general step; short
    wavelengths with weak line opacity put about half the lanes there, mixed inside most
    64-lane waves, so both step forms run in one wave.  Every lane form (one, two and four
    lanes per wavelength; the grouped forms take the contracted table only) against the
    oracle, 3 T-P iterations, contracted and per-species.  ptop = -2 (top of the atmosphere at
    1e-2 bar): the same albedo mix with no optically thin layer — the reference algorithm's
    one-ulp floor 6.6e-13 against 1.6e-10 at 1e-6 bar — held to 1e-10 outright (the
    well-conditioned twin)."""
    rng = np.random.default_rng(41)
    lam, _, _ = O.wavelength_grid(0.3, 3, 2048)
    nL = 20
    p = O.pressure_grid(nL, ptop, np.log10(200))
    T0 = O.temperature_grid(p, 1600.0, 0.1, 0.1)
    Tn = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 6)
    names = ["1H2-16O", "12C-16O"]
    mmr = O.mock_mmr(names, M_BAR)[:, None] * np.ones(nL)
    tabs_o, tabs_f = {}, {}
    for n in names:
        base = 10 ** rng.uniform(-4, 0, lam.size)
        fp, fT = (p / 1.0) ** 0.1, (Tn / 1000.0) ** 0.5
        tabs_o[n] = O.Table(O.separable_table(base, fp, fT), p, Tn)
        tabs_f[n] = fa.SeparableTable(base, fp, fT, p, Tn)
    # the albedo the first sweep sees: a mix, and mixed within waves
    k, sig = O.kappa(tabs_o, T0[5], p[5], lam, M_BAR, mmr=mmr[:, 5])
    w0 = sig / (sig + k)
    frac = (w0 > 0.1).mean()
    mixed = np.mean([0 < (w0[i:i + 64] > 0.1).mean() < 1 for i in range(0, lam.size, 64)])
    assert 0.2 < frac < 0.8 and mixed > 0.5, (frac, mixed)
    cond = _cond((nL, lam.size))
    osp, oT, oth, odt, ou, od, it = O.emission_spectrum(
        tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1, n_timesteps=3,
        n_zero_crossings=10 ** 6, convergence_dT=-1, mmr=mmr, err=cond)
    floor = _floor(lambda: O.emission_spectrum(
        tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1, n_timesteps=3,
        n_zero_crossings=10 ** 6, convergence_dT=-1, mmr=mmr))
    monkeypatch.setenv("FREI_PRECONTRACT", precontract)
    forms = [(1, 0), (2, 0), (4, 0), (1, 1), (1, 2), (1, 4)] if precontract == "1" else [(1, 0)]
    for q, nc in forms:   # lanes per wavelength, producer/consumer sweep's consumers per block
        monkeypatch.setenv("FREI_GROUP_Q", str(q))
        monkeypatch.setenv("FREI_PIPE", str(nc))
        eng = fa.Engine(lam, p, tabs_f, mmr=mmr)
        try:
            path = eng.path()
            assert (path["paired"], path["quad"], path["pipe"]) == (q == 2, q == 4, nc)
            assert path["contracted"] == (precontract == "1")
            r = eng.run(T0, n_timesteps=3, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            up, down = eng.get_fluxes()
        finally:
            eng.close()
        what = f"high albedo Q{q} pipe {nc} precontract {precontract} ptop {ptop}"
        relT = rel(r["final_T"], oT)
        assert relT < 1e-10, (what, relT)
        delta = max(EPS, relT)
        assert_flux_parity(r["spectrum"], osp, cond["up"][-1], delta, what + " spectrum")
        assert_flux_parity(up, ou, cond["up"], delta, what + " F_up")
        assert_flux_parity(down, od, cond["down"], delta, what + " F_down")
        e = assert_grid_parity(r["spectrum"], osp, up, ou, down, od, what, floor,
                               T=r["final_T"], ref_T=oT)
        if ptop == -2:
            assert max(floor) < 1e-11 and e["within_1e-10"], e


@pytest.mark.parametrize("depth,pf", [(2, 8), (2, 16), (4, 8), (4, 16)])
@pytest.mark.parametrize("n_layers", [5, 34, 60])
def test_deep_prefetch_sweep_is_bitwise_the_one_lane_form(fa, monkeypatch, depth, pf, n_layers):
    """FREI_PREFETCH_STEPS: the contracted one-lane sweep with its loads issued 8 or 16 steps
    ahead (a register ring) runs the same arithmetic in the same order, so one sweep each way
    and a T-P run are bit-identical to the default distance (5 layers: fewer steps than the
    ring; 34 / 60: partial last rounds)."""
    rng = np.random.default_rng(19)
    lam, _, _ = O.wavelength_grid(0.5, 10, 3000)
    p = O.pressure_grid(n_layers, -6, np.log10(200))
    T0 = O.temperature_grid(p, 1600.0, 0.1, 0.1)
    Tn = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 9)
    names = ["1H2-16O", "12C-16O"]
    tabs = {n: fa.SeparableTable(10 ** rng.uniform(-4, 2, lam.size), (p / 1.0) ** 0.1,
                                 (Tn / 1000.0) ** 0.5, p, Tn) for n in names}
    mmr = O.mock_mmr(names, M_BAR)[:, None] * np.ones(n_layers)
    monkeypatch.setenv("FREI_GROUP_Q", "1")
    monkeypatch.setenv("FREI_PIPE", "0")
    monkeypatch.setenv("FREI_PREFETCH_DEPTH", str(depth))
    out = {}
    for steps in (0, pf):
        monkeypatch.setenv("FREI_PREFETCH_STEPS", str(steps))
        eng = fa.Engine(lam, p, tabs, mmr=mmr)
        try:
            assert eng.path()["contracted"]
            r = {}
            for d in (0, 1):
                eng.set_temperatures(T0)
                eng.set_fluxes(np.full((n_layers, lam.size), 1e9),
                               np.full((n_layers, lam.size), 2e8))
                r[d] = eng.sweep(d, alpha=1.0) + eng.get_fluxes()
            r["run"] = eng.run(T0, n_timesteps=4, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            out[steps] = r
        finally:
            eng.close()
    a, b = out[pf], out[0]
    for d in (0, 1):
        for x, y in zip(a[d], b[d]):
            assert np.array_equal(x, y), (depth, pf, d)
    for k in ("final_T", "spectrum", "dtaus"):
        assert np.array_equal(a["run"][k], b["run"][k]), k
