"""GPU parity of the batched engine (§8(f) #2, config C5): n_atm atmospheres that differ in
T, gravity and metallicity, on shared wavelengths, pressures and tables, as one device run
(sweeps over (wavelength block, atmosphere), per-atmosphere species contraction on fp64
MFMA).  Each atmosphere is checked against the oracle's emission_spectrum (the reference's
per-Grid loop) under the flux criterion of tests/parity.py, with identical iteration counts
to convergence, and against the single-atmosphere engine."""
import numpy as np
import pytest

from oracle import frei_oracle as O
from tests.parity import (EPS, assert_flux_parity, assert_grid_parity, grid_floor,
                          perturbed_exp, rel, row_normwise)

pytestmark = pytest.mark.gpu

M_BAR = 4.0142926168559996e-24


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    from frei_amd import _native as N
    assert N.device_count() >= 1, "no HIP device visible"
    return frei_amd


def _setup(fa, n_atm, n_lam, n_layers, names, seed):
    rng = np.random.default_rng(seed)
    lam, _, _ = O.wavelength_grid(0.5, 10, n_lam)
    p = O.pressure_grid(n_layers, -6, np.log10(200))
    Tn = np.linspace(400.0, 4000.0, 12)
    tabs_o, tabs_f = {}, {}
    for n in names:
        base = 10 ** rng.uniform(-3, 1.5, lam.size)
        fp, fT = (p / 1.0) ** 0.1, (Tn / 1000.0) ** 0.5
        tabs_o[n] = O.Table(O.separable_table(base, fp, fT), p, Tn)
        tabs_f[n] = fa.SeparableTable(base, fp, fT, p, Tn)
    T_ref = rng.uniform(1100, 2500, n_atm)
    g = rng.uniform(800.0, 6000.0, n_atm)
    mh = rng.uniform(-0.5, 1.0, n_atm)
    mmr0 = O.mock_mmr(names, M_BAR)
    mmr = np.array([(mmr0 * 10 ** m)[:, None] * np.ones(n_layers) for m in mh])
    T0 = np.array([O.temperature_grid(p, t, 0.1, 0.1) for t in T_ref])
    return lam, p, tabs_o, tabs_f, g, mmr, T0


@pytest.mark.parametrize("k7_mfma", ["1", "0"])
def test_batched_atmospheres_match_oracle_per_atmosphere(fa, monkeypatch, k7_mfma):
    monkeypatch.setenv("FREI_K7_MFMA", k7_mfma)   # K7 on MFMA / on the VALU
    names = ["1H2-16O", "12C-16O", "Na"]
    lam, p, tabs_o, tabs_f, g, mmr, T0 = _setup(fa, 5, 2048, 30, names, 17)
    Ft = O.F_TOA(lam)
    eng = fa.BatchEngine(lam, p, tabs_f, g=g, mmr=mmr, F_toa=Ft)
    try:
        assert eng.path()["contracted"]
        out = eng.run(T0, n_timesteps=40, n_zero_crossings=2, convergence_dT=3.0, alpha=1.0)
        ups, downs = eng.get_fluxes()
    finally:
        eng.close()
    for m in range(5):
        cond = dict(up=np.zeros((30, lam.size)), down=np.zeros((30, lam.size)), delta=1.0)
        osp, oT, oth, odt, ou, od, it = O.emission_spectrum(
            tabs_o, T0[m], p, lam, Ft, g[m], M_BAR, 1, n_timesteps=40, n_zero_crossings=2,
            convergence_dT=3.0, mmr=mmr[m], err=cond)
        assert out["n_iter"][m] == it, f"atmosphere {m}: iterations"
        with perturbed_exp():
            psp, pT, _, _, pu, pd, _ = O.emission_spectrum(
                tabs_o, T0[m], p, lam, Ft, g[m], M_BAR, 1, n_timesteps=40, n_zero_crossings=2,
                convergence_dT=3.0, mmr=mmr[m])
        # 40 iterations without meeting the convergence test: one ulp of exp moves the oracle's
        # own T by up to 1.1e-10 here (atmosphere 3), so T is held to 1e-10 or twice that floor
        T_floor = rel(pT, oT)
        relT = rel(out["final_T"][m], oT)
        assert relT <= max(1e-10, 2 * T_floor), f"atmosphere {m}: T {relT:.3e} (floor {T_floor:.3e})"
        assert_flux_parity(out["spectra"][m], osp, cond["up"][-1], max(EPS, relT),
                           f"atmosphere {m} spectrum")
        floor = grid_floor(osp, ou, od, psp, pu, pd)
        assert_grid_parity(out["spectra"][m], osp, ups[m], ou, downs[m], od, f"atmosphere {m}",
                           floor, T=out["final_T"][m], ref_T=oT, T_floor=T_floor)


def test_batched_atmospheres_strong_opacity_at_1e10_outright(fa):
    """The well-conditioned twin of the toy batched atmospheres above: five
    atmospheres on tables of 10-1000 cm^2 g^-1 (no optically thin layer; seed chosen so that no
    layer sits on the convective branch's switch), four fixed T-P iterations through K7 and the
    batched sweeps, each atmosphere against its own oracle run at 1e-10 with no floor rule —
    the reference algorithm's own one-ulp floor here is <= 1.3e-13, asserted too."""
    rng = np.random.default_rng(30)
    names = ["1H2-16O", "12C-16O", "Na"]
    lam, _, _ = O.wavelength_grid(0.5, 10, 2048)
    nL = 30
    p = O.pressure_grid(nL, -6, np.log10(200))
    Tn = np.linspace(400.0, 5000.0, 12)
    tabs_o, tabs_f = {}, {}
    for n in names:
        base = 10 ** rng.uniform(0, 4.5, lam.size)
        fp, fT = (p / 1.0) ** 0.1, (Tn / 1000.0) ** 0.5
        tabs_o[n] = O.Table(O.separable_table(base, fp, fT, 10.0, 1e3), p, Tn)
        tabs_f[n] = fa.SeparableTable(base, fp, fT, p, Tn, lo=10.0, hi=1e3)
    T_ref = rng.uniform(1100, 2500, 5)
    g = rng.uniform(800.0, 6000.0, 5)
    mh = rng.uniform(-0.5, 1.0, 5)
    mmr0 = O.mock_mmr(names, M_BAR)
    mmr = np.array([(mmr0 * 10 ** m)[:, None] * np.ones(nL) for m in mh])
    T0 = np.array([O.temperature_grid(p, t, 0.1, 0.1) for t in T_ref])
    Ft = O.F_TOA(lam)
    eng = fa.BatchEngine(lam, p, tabs_f, g=g, mmr=mmr, F_toa=Ft)
    try:
        assert eng.path()["contracted"]
        out = eng.run(T0, n_timesteps=4, n_zero_crossings=10 ** 6, convergence_dT=-1.0, alpha=1.0)
        ups, downs = eng.get_fluxes()
    finally:
        eng.close()
    for m in range(5):
        run = lambda: O.emission_spectrum(tabs_o, T0[m], p, lam, Ft, g[m], M_BAR, 1,
                                          n_timesteps=4, n_zero_crossings=10 ** 6,
                                          convergence_dT=-1.0, mmr=mmr[m])
        osp, oT, oth, odt, ou, od, it = run()
        with perturbed_exp():
            psp, pT, _, _, pu, pd, _ = run()
        assert max(grid_floor(osp, ou, od, psp, pu, pd)) < 1e-12 and rel(pT, oT) < 1e-12
        e = assert_grid_parity(out["spectra"][m], osp, ups[m], ou, downs[m], od,
                               f"strong atmosphere {m} (outright)", T=out["final_T"][m], ref_T=oT)
        assert e["within_1e-10"], e


@pytest.mark.parametrize("k7_mfma", ["1", "0"])
def test_batched_mfma_contraction_tiles_and_padding(fa, monkeypatch, k7_mfma):
    """17 atmospheres (two 16-row MFMA tiles, one padded) x 5 species (a padded K step):
    fixed-work iterations agree with one single-atmosphere engine per atmosphere (both K7
    forms; the VALU form sums the species in K3's order)."""
    monkeypatch.setenv("FREI_K7_MFMA", k7_mfma)
    names = ["1H2-16O", "12C-16O", "12C-16O2", "Na", "K"]
    lam, p, tabs_o, tabs_f, g, mmr, T0 = _setup(fa, 17, 700, 16, names, 23)
    eng = fa.BatchEngine(lam, p, tabs_f, g=g, mmr=mmr)
    try:
        eng.state_init(T0)
        eng.iterate(3)
        eng.synchronize()
        up, down = eng.get_fluxes()
        import ctypes
        from frei_amd import _native as N
        Tb = np.empty((17, 16))
        N.check(N.lib().frei_get_temperatures(eng._ctx, N.dptr(Tb)))
    finally:
        eng.close()
    monkeypatch.delenv("FREI_K7_MFMA")
    for m in (0, 7, 16):
        single = fa.Engine(lam, p, tabs_f, g=g[m], mmr=mmr[m])
        try:
            single.state_init(T0[m])
            single.iterate(3)
            single.synchronize()
            su, sd = single.get_fluxes()
            Ts = single.get_temperatures()
        finally:
            single.close()
        assert rel(Tb[m], Ts) < 1e-12, f"atmosphere {m}: T"
        assert rel(up[m][-1], su[-1]) < 1e-9, f"atmosphere {m}: emergent F_up"


def test_batched_emission_spectra_over_grids(fa):
    """batched_emission_spectra over Grid objects (a T_ref x g sweep) equals each Grid's own
    emission_spectrum within the parity tolerance, with the same iteration counts."""
    lam, _, _ = O.wavelength_grid(0.5, 10, 1024)
    grids = []
    op = None
    # planets that also differ in their star (T_star) and orbit (a/R_star): each atmosphere
    # gets its own F_TOA
    for T_ref, g, T_star, a_r in [(1400, 1500.0, 5800.0, 6.450964670116429),
                                  (2000, 2478.6519476149147, 4500.0, 5.0),
                                  (2400, 4000.0, 6500.0, 8.0)]:
        pl = fa.Planet.from_hot_jupiter()
        pl.g = g
        pl.T_star = T_star
        pl.a_rstar = a_r
        gr = fa.Grid(pl, lam=lam, n_layers=20, T_ref=T_ref)
        if op is None:
            op = fa.load_example_opacity(gr, scale_factor=2)
        gr.load_opacities(opacities=op)
        grids.append(gr)
    res = fa.batched_emission_spectra(grids, n_timesteps=30)
    tabs_o = {"1H2-16O": O.Table(op["1H2-16O"].values, op["1H2-16O"].pressure,
                                 op["1H2-16O"].temperature)}
    for gr, (spec, T, it) in zip(grids, res):
        s1, T1, th1, _ = gr.emission_spectrum(n_timesteps=30)
        gr._close_engine()
        assert it == th1.shape[1] // 2
        # batch (K7 MFMA contraction) and single (K3) round the species sum differently; both
        # must sit within the reference's own one-ulp floor of the oracle's T and spectrum
        pl = gr.planet
        Ft = O.F_TOA(lam, T_star=pl.T_star, a_rstar=pl.a_rstar)

        def run():
            return O.emission_spectrum(tabs_o, gr.init_temperatures, gr.pressures, lam, Ft, pl.g,
                                       pl.m_bar, pl.alpha, n_timesteps=30)
        osp, oT, *_ = run()
        with perturbed_exp():
            psp, pT, *_ = run()
        fT, fS = rel(pT, oT), rel(psp, osp)
        for t, sp_ in ((T, spec.flux), (T1, s1.flux)):
            assert rel(t, oT) <= max(1e-10, 2 * fT), (rel(t, oT), fT)
            assert rel(sp_, osp) <= max(1e-10, 2 * fS), (rel(sp_, osp), fS)


@pytest.mark.parametrize("nc", [1, 4])
def test_batched_pipe_sweep_matches_one_lane(fa, monkeypatch, nc):
    """The producer/consumer sweep over (wavelength block, atmosphere) launches: with 4
    consumers per block every atmosphere's T, spectrum and fluxes are bitwise those of the
    one-lane sweep; with 1 only the block-sum tree of the bolometric partials differs."""
    names = ["1H2-16O", "12C-16O", "Na"]
    lam, p, tabs_o, tabs_f, g, mmr, T0 = _setup(fa, 3, 3000, 24, names, 23)
    out = {}
    monkeypatch.setenv("FREI_GROUP_Q", "1")
    for v in (0, nc):
        monkeypatch.setenv("FREI_PIPE", str(v))
        eng = fa.BatchEngine(lam, p, tabs_f, g=g, mmr=mmr)
        try:
            path = eng.path()
            assert path["contracted"] and path["pipe"] == v, path
            r = eng.run(T0, n_timesteps=6, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            out[v] = (r, eng.get_fluxes())
        finally:
            eng.close()
    (r0, (u0, d0)), (r1, (u1, d1)) = out[0], out[nc]
    assert np.array_equal(r0["n_iter"], r1["n_iter"])
    if nc == 4:
        assert np.array_equal(r1["final_T"], r0["final_T"])
        assert np.array_equal(r1["spectra"], r0["spectra"])
        assert np.array_equal(u1, u0) and np.array_equal(d1, d0)
    else:
        assert rel(r1["final_T"], r0["final_T"]) < 1e-12
        assert row_normwise(r1["spectra"], r0["spectra"]) < 1e-9


def test_tables_are_ordered_after_device_memory_reuse(fa):
    """Table allocation zeroes the row padding on the context's stream, ordered before the
    device-side table generation: a context whose tables land in memory another context just
    freed gives bitwise the results of a fresh one.  (Round 2 found the padding memset on the
    null stream, unordered with the context's non-blocking stream: it could still be zeroing a
    table the generator had written, which changed C5 runs after other contexts.)"""
    from frei_amd.workloads import c3
    from frei_amd.engine import Engine

    def batch_run():
        w = c3(n_layers=60, n_lam=100_000, n_T=16)
        tabs = {n: fa.SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
                for s, n in enumerate(w["names"])}
        A = 16
        g = np.linspace(300.0, 10000.0, A)
        T0 = np.array([w["T0"] * (0.85 + 0.3 * m / A) for m in range(A)])
        mmr = np.broadcast_to(w["mmr"], (A,) + w["mmr"].shape)
        eng = fa.BatchEngine(w["lam"], w["p"], tabs, g=g, mmr=mmr)
        try:
            return eng.run(T0, n_timesteps=12, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
        finally:
            eng.close()

    fresh = batch_run()
    w3 = c3(n_lam=400_000)   # a large context created, iterated and freed in between
    tabs3 = {n: fa.SeparableTable(w3["base"][s], w3["fp"][s], w3["fT"][s], w3["p"], w3["T_nodes"])
             for s, n in enumerate(w3["names"])}
    e3 = Engine(w3["lam"], w3["p"], tabs3, mmr=w3["mmr"])
    e3.state_init(w3["T0"])
    e3.iterate(3)
    e3.close()
    reused = batch_run()
    assert np.array_equal(fresh["final_T"], reused["final_T"])
    assert np.array_equal(fresh["spectra"], reused["spectra"])


def test_batched_step_records_formed_in_sweep_are_bitwise_the_updates(fa, monkeypatch):
    """In-sweep step records forced on a batched context (FREI_REC_SWEEP=1; off by default for
    batches): every (block, atmosphere) forms its atmosphere's records from that atmosphere's
    T and gravity — bitwise the results of the update-written records."""
    names = ["1H2-16O", "12C-16O", "Na"]
    lam, p, tabs_o, tabs_f, g, mmr, T0 = _setup(fa, 4, 2500, 26, names, 29)
    out = {}
    for rec in ("0", "1"):
        monkeypatch.setenv("FREI_REC_SWEEP", rec)
        eng = fa.BatchEngine(lam, p, tabs_f, g=g, mmr=mmr)
        try:
            assert eng.path()["lds_steps"]
            r = eng.run(T0, n_timesteps=8, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            out[rec] = (r, eng.get_fluxes())
        finally:
            eng.close()
    (a, fa_), (b, fb_) = out["0"], out["1"]
    assert np.array_equal(a["final_T"], b["final_T"])
    assert np.array_equal(a["spectra"], b["spectra"])
    assert all(np.array_equal(x, y) for x, y in zip(fa_, fb_))


def test_batched_two_wavelength_sweep_matches_one_lane(fa, monkeypatch):
    """Two wavelengths per lane over (wavelength block, atmosphere) launches (forced here; the
    C5 size selects it by itself, test_gpu_c5_fullsize.py): every atmosphere's single-sweep
    fluxes are the one-lane sweep's bit for bit, so after a run the temperatures differ only by
    the bolometric summation tree, with equal iteration counts.  That difference is rounding,
    but the deepest layer's dT amplifies it: 2e-11 relative after six iterations here, so the
    bound is the parity bar (1e-10; the oracle pins this form at C5 size in
    test_gpu_c5_fullsize.py)."""
    names = ["1H2-16O", "12C-16O", "Na"]
    lam, p, tabs_o, tabs_f, g, mmr, T0 = _setup(fa, 3, 3000, 24, names, 23)
    out = {}
    monkeypatch.setenv("FREI_GROUP_Q", "1")
    monkeypatch.setenv("FREI_PIPE", "0")
    monkeypatch.setenv("FREI_SHARED", "0")
    for v in (0, 1):
        monkeypatch.setenv("FREI_LAM2", str(v))
        eng = fa.BatchEngine(lam, p, tabs_f, g=g, mmr=mmr)
        try:
            path = eng.path()
            assert path["contracted"] and path["lam2"] == bool(v), path
            r = eng.run(T0, n_timesteps=6, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            out[v] = (r, eng.get_fluxes())
        finally:
            eng.close()
    (r0, _), (r1, _) = out[0], out[1]
    assert np.array_equal(r0["n_iter"], r1["n_iter"])
    assert rel(r1["final_T"], r0["final_T"]) < 1e-10
    assert row_normwise(r1["spectra"], r0["spectra"]) < 1e-9
