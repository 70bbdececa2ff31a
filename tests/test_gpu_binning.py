"""GPU parity of K6, opacity binning (frei/opacity.py:66-170, frei/interp.py:156-307),
through the C ABI, against the reference's own binned_opacity (tests/golden/binning.npz)
and the CPU oracle.

groupies mode (float32 accumulator, sequential pair order): bit-exact.
exact mode (float64 trapezoid integral, then linear interpolation): the NaN pattern of
single-point bins is identical, values agree to 1e-13 relative (the reference's
np.sum may sum a bin pairwise, the kernel sums in point order; all terms are >= 0)."""
import numpy as np
import pytest

from oracle import frei_oracle as O

pytestmark = pytest.mark.gpu

EXACT_RTOL = 1e-13


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    from frei_amd import _native as N
    assert N.device_count() >= 1, "no HIP device visible"
    return frei_amd


@pytest.fixture(scope="module")
def xs(fa, golden):
    B = golden("binning.npz")
    x = fa.CrossSection(B["xsec"], B["xsec_T"], B["xsec_p"], B["xsec_wl"], "1H2-16O")
    yield B, x
    x.release()


def _assert_exact(out, ref, what):
    assert np.array_equal(np.isnan(out), np.isnan(ref)), what + ": NaN pattern"
    ok = ~np.isnan(ref)
    err = np.abs(out[ok] - ref[ok])
    assert np.all(err <= EXACT_RTOL * np.abs(ref[ok])), \
        f"{what}: max rel {np.max(err / np.abs(ref[ok])):.3e}"


@pytest.mark.parametrize("case", ["g1", "g2", "tie"])
def test_groupies_binning_bit_exact_vs_reference(xs, case):
    B, x = xs
    grid = "g1" if case == "tie" else case
    out = x.bin(B[f"{grid}_wl_bins"], B[f"{grid}_lam"], B[f"{case}_T"], B[f"{case}_p"],
                groupies=True)
    ref = np.transpose(B[f"{case}_groupies"], (1, 0, 2))
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("case", ["g1", "g2", "tie"])
def test_exact_binning_matches_reference(xs, case):
    B, x = xs
    grid = "g1" if case == "tie" else case
    out = x.bin(B[f"{grid}_wl_bins"], B[f"{grid}_lam"], B[f"{case}_T"], B[f"{case}_p"],
                groupies=False)
    _assert_exact(out, np.transpose(B[f"{case}_exact"], (2, 1, 0)), case)
    orc = O.binned_opacity(B["xsec"], B["xsec_T"], B["xsec_p"], B["xsec_wl"], B[f"{case}_T"],
                           B[f"{case}_p"], B[f"{grid}_wl_bins"], B[f"{grid}_lam"],
                           groupies=False)
    assert np.array_equal(np.isnan(out), np.isnan(orc))
    ok = ~np.isnan(orc)
    assert np.array_equal(out[ok], orc[ok]), "kernel vs oracle (same summation order)"


def test_random_cross_section_large_grid_matches_oracle(fa):
    """Denser data than the goldens: 3 x 2 source nodes x 300k points onto 50k bins (both
    modes), target nodes with repeated nearest selections (fan-out of one source row to
    several table rows)."""
    rng = np.random.default_rng(11)
    nu = np.linspace(1000.0, 20000.0, 300_001)
    wl = (1e4 / nu)[1:][::-1]
    T_src, p_src = np.array([800.0, 1600.0, 2400.0]), np.array([1e-3, 1.0])
    xsec = (10 ** rng.uniform(-4, 2, (3, 2, wl.size))).astype(np.float32)
    lam, wl_bins, _ = O.wavelength_grid(0.5, 10, 50_000)
    T_t = np.array([700.0, 900.0, 1500.0, 2600.0, 3000.0])
    p_t = np.array([1e-4, 1e-2, 0.8, 5.0])
    x = fa.CrossSection(xsec, T_src, p_src, wl)
    try:
        for groupies in (True, False):
            out = x.bin(wl_bins, lam, T_t, p_t, groupies=groupies)
            ref = O.binned_opacity(xsec, T_src, p_src, wl, T_t, p_t, wl_bins, lam, groupies)
            assert np.array_equal(np.isnan(out), np.isnan(ref))
            ok = ~np.isnan(ref)
            assert np.array_equal(out[ok], ref[ok]), f"groupies={groupies}"
    finally:
        x.release()


def test_grid_bins_into_device_tables_and_runs(fa, golden):
    """Grid.load_opacities(cross_sections=...) bins on the device straight into the engine
    tables; the T-P loop result equals the same run on the host-binned tables uploaded
    with frei_set_table (bitwise), and matches the oracle on the oracle-binned tables."""
    B = golden("binning.npz")
    planet = fa.Planet.from_hot_jupiter()
    for groupies in (True, False):
        grid = fa.Grid(planet, n_layers=6, T_ref=2400)
        x = fa.CrossSection(B["xsec"], B["xsec_T"], B["xsec_p"], B["xsec_wl"], "1H2-16O")
        grid.load_opacities(cross_sections={"1H2-16O": x}, groupies=groupies)
        spec, T, th, dt = grid.emission_spectrum(n_timesteps=3)
        tab = grid.opacities["1H2-16O"]
        host = fa.OpacityTable(tab.values, tab.pressure, tab.temperature)
        # this Grid's own arrays (its logspace grid differs from the golden's by ulps)
        ref_tab = O.binned_opacity(B["xsec"], B["xsec_T"], B["xsec_p"], B["xsec_wl"],
                                   grid.init_temperatures, grid.pressures, grid.wl_bins,
                                   grid.lam, groupies=groupies)
        assert np.array_equal(np.isnan(host.values), np.isnan(ref_tab))
        ok = ~np.isnan(ref_tab)
        assert np.array_equal(host.values[ok], ref_tab[ok])
        grid2 = fa.Grid(planet, n_layers=6, T_ref=2400)
        grid2.load_opacities(opacities={"1H2-16O": host})
        spec2, T2, th2, dt2 = grid2.emission_spectrum(n_timesteps=3)
        assert np.array_equal(T, T2) and np.array_equal(spec.flux, spec2.flux)
        assert np.array_equal(dt, dt2, equal_nan=True)
        grid._close_engine()
        grid2._close_engine()
        x.release()


def test_sharded_binning_matches_whole_grid(fa, golden):
    """A context owning a wavelength slice bins only its slice (exact mode reaches the
    neighbouring groups outside the slice for the interpolation)."""
    B = golden("binning.npz")
    x = fa.CrossSection(B["xsec"], B["xsec_T"], B["xsec_p"], B["xsec_wl"])
    lam, wl_bins = B["g2_lam"], B["g2_wl_bins"]
    T_t, p_t = B["g2_T"], B["g2_p"]
    try:
        for groupies in (True, False):
            whole = x.bin(wl_bins, lam, T_t, p_t, groupies=groupies)
            tab = fa.BinnedTable(x, wl_bins, lam, T_t, p_t, groupies)
            for lo, hi in [(0, 1000), (1000, 3001), (3001, 6000)]:
                eng = fa.Engine(lam, p_t, {"1H2-16O": tab},
                                lam_slice=(lo, hi))
                try:
                    k, _ = eng.kappa(float(T_t[1]), float(p_t[1]))
                finally:
                    eng.close()
                # kappa at an on-node (T, p): mmr * table row + sigma, table row = whole[1, 1]
                eng_w = fa.Engine(lam, p_t, {"1H2-16O": fa.OpacityTable(whole, p_t, T_t)},
                                  lam_slice=(lo, hi))
                try:
                    kw, _ = eng_w.kappa(float(T_t[1]), float(p_t[1]))
                finally:
                    eng_w.close()
                assert np.array_equal(np.isnan(k), np.isnan(kw))
                ok = ~np.isnan(kw)
                assert np.array_equal(k[ok], kw[ok]), (groupies, lo, hi)
    finally:
        x.release()


@pytest.mark.parametrize("n_pts,n_bins", [(300_001, 3000), (100_001, 60_000)])
def test_exact_binning_wide_and_sparse_groups_vs_oracle(fa, n_pts, n_bins):
    """The exact mode's lanes integrate the two bins of their interpolation bracket themselves:
    at 3000 bins over 300k points each bin holds ~100 points (the four-point load batches and
    their tails); at 60k bins over 100k points a fifth of the bins are empty and over a third hold
    one point (brackets between non-adjacent bins, NaN from single-point bins), with one source row fanned out to
    several table rows.  Bit for bit the oracle (same summation order)."""
    rng = np.random.default_rng(12)
    nu = np.linspace(1000.0, 20000.0, n_pts)
    wl = (1e4 / nu)[1:][::-1]
    T_src, p_src = np.array([800.0, 1600.0, 2400.0]), np.array([1e-3, 1.0])
    xsec = (10 ** rng.uniform(-4, 2, (3, 2, wl.size))).astype(np.float32)
    lam, wl_bins, _ = O.wavelength_grid(0.5, 10, n_bins)
    T_t = np.array([700.0, 900.0, 1500.0, 2600.0, 3000.0])
    p_t = np.array([1e-4, 1e-2, 0.8, 5.0])
    x = fa.CrossSection(xsec, T_src, p_src, wl)
    try:
        out = x.bin(wl_bins, lam, T_t, p_t, groupies=False)
    finally:
        x.release()
    ref = O.binned_opacity(xsec, T_src, p_src, wl, T_t, p_t, wl_bins, lam, False)
    assert np.array_equal(np.isnan(out), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.array_equal(out[ok], ref[ok])
    assert ok.mean() > 0.2


def test_plan_buffers_reused_across_grids(fa):
    """The plan arrays stay on the device between calls (grown when a call needs more): binning
    onto a fine grid, a coarse one, the fine one again and then the coarse one in the other mode
    with one CrossSection gives each call's result bit for bit what a fresh CrossSection gives."""
    rng = np.random.default_rng(13)
    nu = np.linspace(1000.0, 20000.0, 200_001)
    wl = (1e4 / nu)[1:][::-1]
    T_src, p_src = np.array([800.0, 1600.0, 2400.0]), np.array([1e-3, 1.0])
    xsec = (10 ** rng.uniform(-4, 2, (3, 2, wl.size))).astype(np.float32)
    fine = O.wavelength_grid(0.5, 10, 40_000)
    coarse = O.wavelength_grid(0.7, 8, 2_500)
    T_t, p_t = np.array([700.0, 1500.0, 2600.0]), np.array([1e-4, 0.8, 5.0])
    calls = [(fine, False), (coarse, False), (fine, False), (coarse, True), (fine, True)]
    x = fa.CrossSection(xsec, T_src, p_src, wl)
    try:
        reused = [x.bin(g[1], g[0], T_t, p_t, groupies=gr) for g, gr in calls]
    finally:
        x.release()
    for (g, gr), out in zip(calls, reused):
        y = fa.CrossSection(xsec, T_src, p_src, wl)
        try:
            fresh = y.bin(g[1], g[0], T_t, p_t, groupies=gr)
        finally:
            y.release()
        assert np.array_equal(out, fresh, equal_nan=True), (g[0].size, gr)


def test_exact_binning_wavelengths_far_from_bin_centres(fa):
    """interp1d takes any ascending wavelengths: here the first 1000 skip ~12 bins each, so a
    block of 256 output wavelengths spans ~3000 bins (96 KiB of integrals in LDS, above the
    64 KiB a launch gets without opting in), and the other 19000 crowd the last 40 % of the bins.
    Bit for bit the oracle."""
    nu = np.linspace(1000.0, 20000.0, 300_001)
    wl = (1e4 / nu)[1:][::-1]
    lam0, wl_bins, _ = O.wavelength_grid(0.5, 10, 20_000)
    lam = np.concatenate([lam0[np.linspace(0, 11999, 1000).astype(int)],
                          np.linspace(lam0[12000], lam0[-1], 19000)])
    rng = np.random.default_rng(14)
    T_src, p_src = np.array([800.0, 1600.0]), np.array([1e-3, 1.0])
    xsec = (10 ** rng.uniform(-4, 2, (2, 2, wl.size))).astype(np.float32)
    T_t, p_t = np.array([900.0, 1500.0]), np.array([1e-2, 0.8])
    x = fa.CrossSection(xsec, T_src, p_src, wl)
    try:
        out = x.bin(wl_bins, lam, T_t, p_t, groupies=False)
    finally:
        x.release()
    ref = O.binned_opacity(xsec, T_src, p_src, wl, T_t, p_t, wl_bins, lam, False)
    assert np.isfinite(ref).all()
    assert np.array_equal(out, ref)


def test_exact_binning_unsorted_wavelengths(fa):
    """scipy's interp1d takes the output wavelengths in any order: a shuffled
    wavelength grid gives each wavelength the value the sorted grid gives it — each block's LDS
    window runs from the smallest to the largest bracket of its lanes.  Bit for bit the oracle."""
    nu = np.linspace(1000.0, 20000.0, 200_001)
    wl = (1e4 / nu)[1:][::-1]
    lam0, wl_bins, _ = O.wavelength_grid(0.5, 10, 8_000)
    rng = np.random.default_rng(15)
    perm = rng.permutation(lam0.size)
    lam = lam0[perm]
    T_src, p_src = np.array([800.0, 1600.0]), np.array([1e-3, 1.0])
    xsec = (10 ** rng.uniform(-4, 2, (2, 2, wl.size))).astype(np.float32)
    T_t, p_t = np.array([900.0, 1500.0]), np.array([1e-2, 0.8])
    x = fa.CrossSection(xsec, T_src, p_src, wl)
    try:
        out = x.bin(wl_bins, lam, T_t, p_t, groupies=False)
        out_sorted = x.bin(wl_bins, lam0, T_t, p_t, groupies=False)
    finally:
        x.release()
    ref = O.binned_opacity(xsec, T_src, p_src, wl, T_t, p_t, wl_bins, lam, False)
    assert np.array_equal(out, ref, equal_nan=True)
    assert np.array_equal(out, out_sorted[..., perm], equal_nan=True)


def test_exact_binning_sparse_wavelengths_per_lane_brackets(fa):
    """The first 300 of 60k output wavelengths skip ~100 bins each, so the first block of 256
    spans ~25,600 bins, far more than its LDS window holds (5120): such blocks interpolate lane by lane (each lane integrates its own two
    bins) instead of failing.  Bit for bit the oracle, mixed with dense blocks."""
    nu = np.linspace(1000.0, 20000.0, 240_001)
    wl = (1e4 / nu)[1:][::-1]
    lam0, wl_bins, _ = O.wavelength_grid(0.5, 10, 60_000)
    lam = np.concatenate([lam0[np.linspace(0, 29999, 300).astype(int)],
                          np.linspace(lam0[30000], lam0[-1], lam0.size - 300)])
    rng = np.random.default_rng(16)
    T_src, p_src = np.array([800.0, 1600.0]), np.array([1e-3, 1.0])
    xsec = (10 ** rng.uniform(-4, 2, (2, 2, wl.size))).astype(np.float32)
    T_t, p_t = np.array([900.0, 1500.0]), np.array([1e-2, 0.8])
    x = fa.CrossSection(xsec, T_src, p_src, wl)
    try:
        out = x.bin(wl_bins, lam, T_t, p_t, groupies=False)
    finally:
        x.release()
    ref = O.binned_opacity(xsec, T_src, p_src, wl, T_t, p_t, wl_bins, lam, False)
    assert np.array_equal(out, ref, equal_nan=True)
    assert np.isfinite(ref[..., :300]).all()   # the per-lane blocks are all finite values
