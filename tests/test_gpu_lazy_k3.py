"""Lazy species contraction (option ``lazy_k3``, FREI_LAZY_K3, round 6): with the
two-wavelength sweep the setup contracts no (pressure row, T node) row of the K3 table; the step
records carry a mask of their two rows not contracted yet, the sweep contracts those for each
lane's own wavelengths first (contract_kernel's sum, species in order) and the update after it
marks them.  The table values are K3's, so every output is bit-identical to the table contracted
up front: single sweeps, fixed iterations and runs to radiative equilibrium whose temperatures
cross T nodes, a layer outside the table's T hull, and a form change mid-life (the whole table
is contracted before any other sweep form runs)."""
import numpy as np
import pytest

import oracle.frei_oracle as O

pytestmark = pytest.mark.gpu

M_BAR = 4.0142926168559996e-24


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    return frei_amd


def _case(fa, nL=40, n_lam=8192, seed=5, hull=(0.8, 1.2)):
    rng = np.random.default_rng(seed)
    lam, _, _ = O.wavelength_grid(0.5, 10, n_lam)
    p = O.pressure_grid(nL, -6, np.log10(200))
    T0 = O.temperature_grid(p, 1800.0, 0.1, 0.1)
    Tn = np.linspace(hull[0] * T0.min(), hull[1] * T0.max(), 16)
    names = ["1H2-16O", "12C-16O", "12C-1H4", "Na"]
    tabs = {n: fa.SeparableTable(10 ** rng.uniform(-3, 1.5, lam.size), (p / 1.0) ** 0.1,
                                 (Tn / 1000.0) ** 0.5, p, Tn) for n in names}
    mmr = O.mock_mmr(names, M_BAR)[:, None] * np.ones(nL)
    return lam, p, T0, tabs, mmr


def _lam2(eng):
    """The two-wavelength sweep on this small grid (test_gpu_converged_skip's options)."""
    for k, v in (("group_q", 1), ("shared", 0), ("pipe", 0), ("lam2", 1)):
        eng.set_option(k, v)


def _exercise(eng, T0, nL, n_lam):
    rng = np.random.default_rng(9)
    r = {}
    for d in (0, 1):
        eng.set_temperatures(T0 * (1.0 + 0.05 * d))
        eng.set_fluxes(10 ** rng.uniform(8, 12, (nL, n_lam)), 10 ** rng.uniform(6, 11, (nL, n_lam)))
        r[d] = eng.sweep(d, alpha=1.0) + eng.get_fluxes() + (eng.get_temperatures(),)
    r["run"] = eng.run(T0, n_timesteps=200, n_zero_crossings=2, convergence_dT=3.0)
    r["run2"] = eng.run(T0 * 0.9, n_timesteps=7, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
    eng.state_init(T0 * 1.1)
    eng.iterate(6, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
    eng.synchronize()
    r["iterate"] = eng.get_temperatures()
    r["fluxes"] = eng.get_fluxes()
    return r


def _compare(a, b, tag):
    same = lambda x, y, w: np.testing.assert_array_equal(np.asarray(x), np.asarray(y), err_msg=w)
    for d in (0, 1):
        for i, what in enumerate(("dT", "bolometric", "dtaus", "F_up", "F_down", "T")):
            same(a[d][i], b[d][i], f"{tag} dir {d} {what}")
    for key in ("run", "run2"):
        assert a[key]["n_iter"] == b[key]["n_iter"], tag
        for what in ("final_T", "temp_hist", "spectrum", "dtaus"):
            same(a[key][what], b[key][what], f"{tag} {key} {what}")
    same(a["iterate"], b["iterate"], f"{tag} iterate T")
    for i in (0, 1):
        same(a["fluxes"][i], b["fluxes"][i], f"{tag} iterate fluxes")


@pytest.mark.parametrize("hull", [(0.8, 1.2), (1.05, 1.2)])
def test_lazy_contraction_is_bitwise_the_full_table(fa, hull):
    """hull (1.05, 1.2): the coolest layers sit below the lowest T node (fill 0: zero weights on
    rows 0 and 1, which the lazy table holds as zeros)."""
    lam, p, T0, tabs, mmr = _case(fa, hull=hull)
    out, paths = {}, {}
    for lazy in (1, 0):
        eng = fa.Engine(lam, p, tabs, mmr=mmr)
        try:
            _lam2(eng)
            eng.set_option("lazy_k3", lazy)
            paths[lazy] = eng.path()
            out[lazy] = _exercise(eng, T0, len(p), lam.size)
        finally:
            eng.close()
    assert paths[1]["lam2"] and paths[1]["lazy_k3"] and paths[1]["contracted"], paths[1]
    assert not paths[0]["lazy_k3"]
    _compare(out[1], out[0], f"lazy vs full, hull {hull}")
    assert 1 < out[1]["run"]["n_iter"] < 200


def test_lazy_then_other_form_contracts_the_rest(fa):
    """A lazy context that later runs another sweep form (option change, or a sweep outside the
    fused update) contracts every remaining row first: the same numbers as a fully contracted
    context running that form throughout."""
    lam, p, T0, tabs, mmr = _case(fa)
    res = {}
    for lazy in (1, 0):
        eng = fa.Engine(lam, p, tabs, mmr=mmr)
        try:
            _lam2(eng)
            eng.set_option("lazy_k3", lazy)
            eng.run(T0, n_timesteps=3, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            eng.set_option("fused_update", 0)   # reduce + update in two kernels: no marking
            r = eng.run(T0 * 1.05, n_timesteps=3, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            res[lazy] = (r, eng.get_fluxes())
        finally:
            eng.close()
    for k in ("final_T", "spectrum", "dtaus"):
        np.testing.assert_array_equal(res[1][0][k], res[0][0][k], err_msg=k)
    for i in (0, 1):
        np.testing.assert_array_equal(res[1][1][i], res[0][1][i])
