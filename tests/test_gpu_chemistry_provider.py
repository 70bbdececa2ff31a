"""The drop-in honours the caller's chemistry (VERDICT r03 "missing" #1 / "next" #2).

The reference's kappa calls ``chemistry(T, p, opacities.keys(), m_bar=m_bar)`` for every layer
of every sweep (opacity.py:246-248); in its own CI that is FastChem (chemistry.py:142-205).  The
engine takes such a provider as ``chemistry=`` (Grid.load_opacities, Engine, the emit/absorb/
kappa shims; INTEGRATION.md passes frei's own).  Here a fake, strongly T- and p-dependent
provider on the reference's call signature stands in for FastChem (FastChem itself is
third-party and absent: its parity is unpinned); the oracle gets the same provider as its
per-layer ``mmr(T, p)``.  The tests show that the provider's values — not the mock's VMR
1.5e-3 — reach the opacity sum, on every entry point, and that the reference's own mock used as
a provider takes the device-resident T-P loop bit for bit.
"""
import numpy as np
import pytest

from oracle import frei_oracle as O
from tests.parity import assert_grid_parity, grid_floor, perturbed_exp, rel

pytestmark = pytest.mark.gpu

G_J, M_BAR = 2478.6519476149147, 4.0142926168559996e-24
NAMES = ["1H2-16O", "12C-16O", "12C-1H4"]


class FakeFastChem:
    """chemistry(temperatures, pressures, species, return_vmr=False, m_bar=...) ->
    {isotopologue: mmr array}, like frei.chemistry.chemistry: CO rises and CH4 falls with T
    (the CO/CH4 switch FastChem gives a hot Jupiter), H2O tracks p.  Accepts Quantities or
    plain arrays; counts its calls."""

    def __init__(self):
        self.calls = 0

    def __call__(self, temperatures, pressures, species, return_vmr=False, m_bar=None):
        self.calls += 1
        T = np.atleast_1d(np.asarray(getattr(temperatures, "value", temperatures), dtype=float))
        p = np.atleast_1d(np.asarray(getattr(pressures, "value", pressures), dtype=float))
        x = np.tanh((T - 1400.0) / 300.0)
        base = O.mock_mmr(NAMES, M_BAR)
        f = {"1H2-16O": 2.0 * (p / 1.0) ** 0.05,
             "12C-16O": 10 ** (0.9 * x),
             "12C-1H4": 10 ** (-0.9 * x)}
        return {n: base[NAMES.index(n)] * f[n] for n in species}


def oracle_mmr(provider):
    """The oracle's per-layer mmr(T, p) (scalars) from the same provider."""
    def f(T, p):
        out = provider(np.array([T]), np.array([p]), NAMES, m_bar=M_BAR)
        return np.array([out[n][0] for n in NAMES])
    return f


def _case(n_lam=600, nL=30, T_ref=1600.0, log_lo=-3.0, log_hi=1.0):
    """Tables 10^U(log_lo, log_hi) cm^2/g x (p/bar)^0.1 x (T/1000 K)^0.5 on 11 T nodes.  The
    default range leaves the top layers nearly transparent (dtau ~ 1e-7: one ulp of exp moves
    the spectrum by 2.4e-8); log 1..3 is the well-conditioned case (one-ulp floor ~1e-12)."""
    rng = np.random.default_rng(19)
    lam, _, _ = O.wavelength_grid(0.5, 10, n_lam)
    p = O.pressure_grid(nL, -6, np.log10(200))
    T0 = O.temperature_grid(p, T_ref, 0.1, 0.1)
    Tn = np.linspace(0.6 * T0.min(), 1.4 * T0.max(), 11)
    tabs_o, base = {}, {}
    for n in NAMES:
        base[n] = 10 ** rng.uniform(log_lo, log_hi, lam.size)
        tabs_o[n] = O.Table(O.separable_table(base[n], (p / 1.0) ** 0.1, (Tn / 1000.0) ** 0.5),
                            p, Tn)
    return lam, p, T0, Tn, base, tabs_o


def _tabs_f(fa, p, Tn, base):
    return {n: fa.SeparableTable(base[n], (p / 1.0) ** 0.1, (Tn / 1000.0) ** 0.5, p, Tn)
            for n in NAMES}


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    return frei_amd


def test_grid_feeds_the_provider_to_radiative_equilibrium(fa):
    """Grid.load_opacities(chemistry=provider) -> emission_spectrum to convergence: the same
    iterations, spectrum, fluxes and T as the oracle driven by that provider — and far from
    the run the mock chemistry gives."""
    lam, p, T0, Tn, base, tabs_o = _case()
    prov = FakeFastChem()
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), lam=lam, pressures=p, init_temperatures=T0)
    grid.load_opacities(opacities=_tabs_f(fa, p, Tn, base), chemistry=prov)
    spec, T, th, dtaus = grid.emission_spectrum(n_timesteps=60)
    eng = grid.engine()
    assert eng.provider is prov and not eng.path()["contracted"]
    up, down = eng.get_fluxes()
    n_calls = prov.calls
    mock = fa.Grid(fa.Planet.from_hot_jupiter(), lam=lam, pressures=p, init_temperatures=T0)
    mock.load_opacities(opacities=_tabs_f(fa, p, Tn, base))
    mspec, mT, _, _ = mock.emission_spectrum(n_timesteps=60)

    def run():
        return O.emission_spectrum(tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1,
                                   n_timesteps=60, mmr=oracle_mmr(FakeFastChem()))
    osp, oT, oth, odt, ou, od, it = run()
    with perturbed_exp():
        psp, pT, pth, pdt, pu, pd, _ = run()
    assert th.shape[1] == 2 * it, "iterations to convergence"
    assert 2 < it < 60
    # T feeds back through the provider (T -> mixing ratios -> kappa -> fluxes -> dT), so T is
    # held, like tests/test_gpu_parity.py's T-dependent chemistry, to 1e-10 or twice what one ulp
    # of exp moves the oracle's own T on these inputs
    t_floor = max(rel(pT, oT), rel(pth, oth))
    assert_grid_parity(spec.flux, osp, up, ou, down, od, "chemistry provider (Grid)",
                       grid_floor(osp, ou, od, psp, pu, pd))
    assert rel(T, oT) <= max(1e-10, 2 * t_floor), (rel(T, oT), t_floor)
    assert rel(th, oth) <= max(1e-10, 2 * t_floor), (rel(th, oth), t_floor)
    # dtaus follow T through the provider's mixing ratios: their own one-ulp floor
    assert rel(dtaus, odt) <= max(1e-10, 2 * rel(pdt, odt)), (rel(dtaus, odt), rel(pdt, odt))
    # one provider call per sweep (2 per iteration + the final emit) after the T probe
    assert n_calls >= 2 * it + 1
    # the provider's values, not the mock's, reached kappa
    assert rel(mspec.flux, osp) > 1e-3 and rel(mT, oT) > 1e-3


class BumpedFastChem(FakeFastChem):
    """The same provider with CO's mass mixing ratio 1e-8 (relative) higher."""

    def __call__(self, *a, **k):
        out = super().__call__(*a, **k)
        out["12C-16O"] = out["12C-16O"] * (1 + 1e-8)
        return out


def test_provider_radiative_equilibrium_at_1e10_outright(fa):
    """VERDICT r04 "next" #2: the provider path on a well-conditioned atmosphere (opacities
    10-1000 cm^2/g: the oracle's own one-ulp floor <= 1e-10 on every output), held to 1e-10 with
    no floor widening — spectrum elementwise, F_up / F_down row-normwise, T, T history and dtaus
    elementwise, equal iteration counts — and the criterion has teeth: the oracle with one
    species' mmr moved by 1e-8 is rejected."""
    lam, p, T0, Tn, base, tabs_o = _case(log_lo=1.0, log_hi=3.0)
    prov = FakeFastChem()
    grid = fa.Grid(fa.Planet.from_hot_jupiter(), lam=lam, pressures=p, init_temperatures=T0)
    grid.load_opacities(opacities=_tabs_f(fa, p, Tn, base), chemistry=prov)
    spec, T, th, dtaus = grid.emission_spectrum(n_timesteps=60)
    eng = grid.engine()
    assert eng.provider is prov and not eng.path()["contracted"]
    up, down = eng.get_fluxes()
    assert np.array_equal(eng.get_spectrum(), up[-1])      # frei_get_spectrum: one row

    def run(provider):
        return O.emission_spectrum(tabs_o, T0, p, lam, O.F_TOA(lam), G_J, M_BAR, 1,
                                   n_timesteps=60, mmr=oracle_mmr(provider))
    osp, oT, oth, odt, ou, od, it = run(FakeFastChem())
    with perturbed_exp():
        psp, pT, pth, pdt, pu, pd, _ = run(FakeFastChem())
    floor = grid_floor(osp, ou, od, psp, pu, pd)
    assert max(floor) <= 1e-10 and rel(pT, oT) <= 1e-10 and rel(pdt, odt) <= 1e-10, floor
    assert th.shape[1] == 2 * it and 2 < it < 60, "iterations to convergence"
    assert_grid_parity(spec.flux, osp, up, ou, down, od, "chemistry provider, well conditioned",
                       T=T, ref_T=oT)                       # no floor: 1e-10 outright
    assert rel(th, oth) <= 1e-10 and rel(dtaus, odt) <= 1e-10, (rel(th, oth), rel(dtaus, odt))
    bsp, bT, _, _, bu, bd, _ = run(BumpedFastChem())
    assert max(rel(spec.flux, bsp), rel(T, bT)) > 1e-10    # a 1e-8 mmr error would fail
    assert rel(bsp, osp) > 1e-9


def test_reference_mock_as_provider_keeps_the_device_loop(fa):
    """frei's own chemistry (the mock VMR 1.5e-3 when pyfastchem is absent) passed as the
    provider is T-independent: the engine fixes the per-layer mmr once and runs the contracted,
    device-resident T-P loop — bitwise the default run."""
    from frei_amd.chemistry import chemistry as frei_chemistry
    lam, p, T0, Tn, base, _ = _case()
    out = {}
    for chem in (None, frei_chemistry):
        grid = fa.Grid(fa.Planet.from_hot_jupiter(), lam=lam, pressures=p, init_temperatures=T0)
        grid.load_opacities(opacities=_tabs_f(fa, p, Tn, base), chemistry=chem)
        out[chem is None] = grid.emission_spectrum(n_timesteps=40)
        eng = grid.engine()
        assert eng.provider is None and eng.path()["contracted"]
    for a, b in zip(out[True], out[False]):
        a = getattr(a, "flux", a)
        b = getattr(b, "flux", b)
        assert np.array_equal(a, b)


def test_emit_absorb_and_kappa_shims_call_the_provider(fa):
    """The reference's seam functions with a provider: each sweep's kappa uses the provider at
    that sweep's temperatures (Q11: T is updated after the sweep), kappa at the query point."""
    lam, p, T0, Tn, base, tabs_o = _case(n_lam=400, nL=20)
    tabs_f = _tabs_f(fa, p, Tn, base)
    prov = FakeFastChem()
    Ft = O.F_TOA(lam)
    up_f, down_f, T_f, hist_f, dt_f, dT_f = fa.emit(tabs_f, T0, p, lam, Ft, G_J, M_BAR,
                                                    n_timesteps=3, convergence_thresh=-1.0,
                                                    chemistry=prov)
    spec_emit = up_f[-1].copy()    # absorb below updates up_f in place (twostream.py:547-550)
    up_a, down_a, T_a, _, _, dT_a = fa.absorb(tabs_f, T_f, p, lam, Ft, G_J, M_BAR, n_timesteps=1,
                                              fluxes_up=up_f, fluxes_down=down_f,
                                              chemistry=prov)
    mm = oracle_mmr(FakeFastChem())
    T = T0.copy()
    F_up = np.zeros((p.size, lam.size))
    F_down = np.zeros((p.size, lam.size))
    F_down[-1] = Ft
    for _ in range(3):
        F_up, F_down, T = O.emit(tabs_o, T, p, lam, Ft, G_J, M_BAR, 1, F_up, F_down,
                                 mmr=mm)[:3]
    assert rel(T_f, T) < 1e-10
    assert rel(spec_emit, F_up[-1]) < 1e-9      # one-ulp floor of the oracle here: 3.3e-11
    F_up, F_down, T2 = O.absorb(tabs_o, T, p, lam, Ft, G_J, M_BAR, 1, F_up, F_down, mmr=mm)[:3]
    assert rel(T_a, T2) < 1e-10
    assert np.max(np.abs(up_a - F_up)) <= 1e-9 * np.max(np.abs(F_up))
    for Tq, pq in ((T0[4] * 1.2, p[4]), (900.0, np.sqrt(p[9] * p[10]))):
        k, _ = fa.kappa(tabs_f, Tq, pq, lam, M_BAR, chemistry=prov)
        ko, _ = O.kappa(tabs_o, Tq, pq, lam, M_BAR, mmr=mm(Tq, pq))
        km, _ = fa.kappa(tabs_f, Tq, pq, lam, M_BAR)       # the mock
        assert rel(k, ko) < 1e-13
        assert rel(km, ko) > 1e-3
