"""Sweeps and updates launched after the run has converged change nothing.  The convergence flag
is read with a launch's first loads and tested only before its first store (frei_kernels.hip:
sweep_pair_kernel, sweep_pipe_body, update_fused_body), so a converged launch must still return
without writing fluxes, partial sums or temperatures.  A fixed-work batch that stops on
convergence (frei_iterate with a convergence test) runs its remaining iterations as such
launches: 120 and 200 iterations must leave the same temperatures and fluxes, bit for bit, on the
two-wavelength, producer/consumer and one-lane sweep forms."""
import numpy as np
import pytest

import oracle.frei_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    return frei_amd


def _case(fa, nL=30, n_lam=9000):
    rng = np.random.default_rng(17)
    lam, _, _ = O.wavelength_grid(0.5, 10, n_lam)
    p = O.pressure_grid(nL, -6, np.log10(200))
    T0 = O.temperature_grid(p, 2000.0, 0.1, 0.1)
    Tn = np.linspace(0.7 * T0.min(), 1.3 * T0.max(), 9)
    names = ["1H2-16O", "12C-16O"]
    tabs = {n: fa.SeparableTable(10 ** rng.uniform(-3, 1, lam.size), (p / 1.0) ** 0.1,
                                 (Tn / 1000.0) ** 0.5, p, Tn) for n in names}
    return lam, p, T0, tabs


FORMS = {
    "lam2": {"group_q": 1, "shared": 0, "lam2": 1},
    "pipe": {"group_q": 1, "pipe": 4},
    "one_lane": {"group_q": 1, "lam2": 0, "pipe": 0},
}


@pytest.mark.parametrize("form", sorted(FORMS))
def test_launches_after_convergence_change_nothing(fa, form):
    lam, p, T0, tabs = _case(fa)
    eng = fa.Engine(lam, p, tabs)
    out = {}
    try:
        for k, v in FORMS[form].items():
            eng.set_option(k, v)
        n_conv = eng.run(T0, n_timesteps=120, want_dtaus=False)["n_iter"]
        assert 1 < n_conv < 120, n_conv
        for n in (120, 200):
            eng.state_init(T0)
            eng.iterate(n, n_zero_crossings=2, convergence_dT=3.0)
            eng.synchronize()
            out[n] = (eng.get_temperatures(), eng.get_fluxes())
        path = eng.path()
        # the same batch without a convergence test keeps changing T: the runs above did stop
        eng.state_init(T0)
        eng.iterate(120)
        eng.synchronize()
        T_free = eng.get_temperatures()
    finally:
        eng.close()
    assert path["contracted"]
    if form == "lam2":
        assert path["lam2"]
    if form == "pipe":
        assert path["pipe"] == 4
    if form == "one_lane":
        assert not path["lam2"] and path["pipe"] == 0
    assert not np.array_equal(out[120][0], T_free)
    assert np.array_equal(out[120][0], out[200][0])
    for i in (0, 1):
        assert np.array_equal(out[120][1][i], out[200][1][i])
