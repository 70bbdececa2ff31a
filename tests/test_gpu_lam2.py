"""Two wavelengths per lane (frei_kernels.hip sweep_pair_kernel, option ``lam2``) against the
one-lane contracted sweep it replaces on large slices.  Every wavelength's flux recurrence is
the one-lane form's expression for expression, so single-sweep fluxes and dtaus must agree bit
for bit; the bolometric partial sums follow this form's own fixed tree (the lane adds its two
wavelengths' weighted terms first), so the sums agree to 1e-13 and the temperatures to 1e-12,
per sweep and over whole runs, with the same iteration counts; the emergent spectrum, which is
ill-conditioned in thin layers, within 1e-9 of the one-lane run.  The oracle side of
this form is pinned at BASELINE size by test_gpu_radeq_fullsize.py / test_gpu_fullsize.py,
where the automatic choice selects it (asserted here through the path report)."""
import numpy as np
import pytest

import oracle.frei_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    return frei_amd


def _rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


def _engine(fa, n_lam, nL=30, seed=57):
    rng = np.random.default_rng(seed)
    lam, _, _ = O.wavelength_grid(0.5, 10, n_lam)
    p = O.pressure_grid(nL, -6, np.log10(200))
    T0 = O.temperature_grid(p, 2200.0, 0.1, 0.1)
    names = ["1H2-16O", "12C-16O", "12C-1H4"]
    Tn = np.linspace(0.7 * T0.min(), 1.3 * T0.max(), 9)
    tabs = {n: fa.SeparableTable(10 ** rng.uniform(-3, 1, lam.size), (p / 1.0) ** 0.1,
                                 (Tn / 1000.0) ** 0.5, p, Tn) for n in names}
    return fa.Engine(lam, p, tabs), p, T0


@pytest.mark.parametrize("n_lam", [5000, 5120, 1026])
def test_two_wavelengths_per_lane_match_one_lane(fa, n_lam):
    eng, p, T0 = _engine(fa, n_lam)
    rng = np.random.default_rng(3)
    up0 = 10 ** rng.uniform(8, 12, (p.size, n_lam))
    dn0 = 10 ** rng.uniform(6, 11, (p.size, n_lam))
    out = {}
    try:
        # the one-lane form with global step records (small slices would otherwise pick the
        # grouped-lane sweep and LDS step tables)
        eng.set_option("group_q", 1)
        eng.set_option("shared", 0)
        for lam2 in (1, 0):
            eng.set_option("lam2", lam2)
            path = eng.path()
            assert path["contracted"] and path["lam2"] == bool(lam2), path
            r = {}
            for d in (0, 1):
                eng.set_temperatures(T0)
                eng.set_fluxes(up0, dn0)
                r[d] = eng.sweep(d, alpha=1.0) + eng.get_fluxes() + (eng.get_temperatures(),)
            r["run"] = eng.run(T0, n_timesteps=80)
            out[lam2] = r
    finally:
        eng.close()
    a, b = out[1], out[0]
    for d in (0, 1):
        dT, bol, dtaus, Fu, Fd, T = range(6)
        for i, what in ((dtaus, "dtaus"), (Fu, "F_up"), (Fd, "F_down")):
            assert np.array_equal(a[d][i], b[d][i]), f"dir {d} {what}"
        err = np.max(np.abs(a[d][bol] - b[d][bol]), axis=0) / np.max(np.abs(b[d][bol]), axis=0)
        assert np.all(err < 1e-13), f"dir {d} bolometric {err}"
        assert _rel(a[d][T], b[d][T]) < 1e-12, f"dir {d} T"
    ra, rb = a["run"], b["run"]
    assert ra["n_iter"] == rb["n_iter"] and 1 < ra["n_iter"] <= 80
    assert _rel(ra["final_T"], rb["final_T"]) < 1e-12
    # the emergent spectrum is ill-conditioned in thin layers (one ulp of exp moves single
    # elements by ~1e-7): 1e-13 in T moves it by up to ~1e-10 here
    assert _rel(ra["spectrum"], rb["spectrum"]) < 1e-9


def test_odd_grid_and_options_fall_back_to_one_lane(fa):
    """An odd wavelength count (no 16-byte pairs) and shared step tables keep the one-lane form."""
    eng, p, T0 = _engine(fa, 5001)
    try:
        eng.set_option("group_q", 1)
        eng.set_option("shared", 0)
        eng.set_option("lam2", 1)
        assert not eng.path()["lam2"]
        r = eng.run(T0, n_timesteps=5)
        assert np.all(np.isfinite(r["final_T"]))
    finally:
        eng.close()
    eng, p, T0 = _engine(fa, 5000)
    try:
        eng.set_option("group_q", 1)
        eng.set_option("lam2", 1)
        eng.set_option("shared", 1)
        assert not eng.path()["lam2"]
    finally:
        eng.close()


def test_auto_selects_two_wavelengths_on_the_500k_grid(fa):
    """The automatic choice at BASELINE's per-GPU size (1954 one-lane blocks) and not at the
    8-GPU slice (245 blocks)."""
    for n_lam, want in ((500_000, True), (62_500, False)):
        eng, p, T0 = _engine(fa, n_lam, nL=8)
        try:
            assert eng.path()["lam2"] == want, n_lam
        finally:
            eng.close()
