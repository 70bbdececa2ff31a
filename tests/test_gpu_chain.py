"""Chained launches (option ``chain``, FREI_CHAIN): each T-P sweep's fused update is deferred
and runs as the leading workgroups of the next sweep's launch, whose sweep blocks poll the
temperatures it publishes (frei_kernels.hip sweep_chain_kernel, stage_records).  The update and
the sweep run the same code as in separate launches, so every output must be bit-identical:
single sweeps, fixed-count iterations, runs to convergence (the converged flag then crosses a
chained launch) — on the grouped-lane paths (two and four lanes per wavelength, 4- and 8-wave
blocks) and the one-lane path (two or four steps in flight), odd and even layer counts, and with
the one-rank P2P exchange in the update."""
import numpy as np
import pytest

import oracle.frei_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    return frei_amd


def _case(fa, nL):
    rng = np.random.default_rng(71)
    lam, _, _ = O.wavelength_grid(0.5, 10, 5000)
    p = O.pressure_grid(nL, -6, np.log10(200))
    T0 = O.temperature_grid(p, 2000.0, 0.1, 0.1)
    Tn = np.linspace(0.7 * T0.min(), 1.3 * T0.max(), 9)
    names = ["1H2-16O", "12C-16O", "12C-1H4"]
    tabs = {n: fa.SeparableTable(10 ** rng.uniform(-3, 1, lam.size), (p / 1.0) ** 0.1,
                                 (Tn / 1000.0) ** 0.5, p, Tn) for n in names}
    return lam, p, T0, tabs


def _exercise(eng, T0, nL, n_lam):
    rng = np.random.default_rng(5)
    r = {}
    for d in (0, 1):
        eng.set_temperatures(T0)
        eng.set_fluxes(10 ** rng.uniform(8, 12, (nL, n_lam)), 10 ** rng.uniform(6, 11, (nL, n_lam)))
        r[d] = eng.sweep(d, alpha=1.0) + eng.get_fluxes() + (eng.get_temperatures(),)
    r["run"] = eng.run(T0, n_timesteps=80)
    r["run2"] = eng.run(T0, n_timesteps=6, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
    eng.state_init(T0)
    eng.iterate(7, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
    eng.synchronize()
    r["iterate"] = eng.get_temperatures()
    r["fluxes"] = eng.get_fluxes()
    return r


def _same(a, b, what):
    assert np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True), what


def _compare(a, b, tag):
    for d in (0, 1):
        for i, what in enumerate(("dT", "bolometric", "dtaus", "F_up", "F_down", "T")):
            _same(a[d][i], b[d][i], f"{tag} dir {d} {what}")
    for key in ("run", "run2"):
        assert a[key]["n_iter"] == b[key]["n_iter"], tag
        for what in ("final_T", "temp_hist", "spectrum", "dtaus"):
            _same(a[key][what], b[key][what], f"{tag} {key} {what}")
    _same(a["iterate"], b["iterate"], f"{tag} iterate T")
    for i in (0, 1):
        _same(a["fluxes"][i], b["fluxes"][i], f"{tag} iterate fluxes")


@pytest.mark.parametrize("nL", [30, 31])
@pytest.mark.parametrize("q,waves,depth", [(2, 4, 0), (2, 8, 0), (4, 4, 0), (4, 8, 0),
                                           (1, 4, 2), (1, 4, 4), (1, 4, "pipe")])
def test_chained_launches_are_bitwise_identical(fa, nL, q, waves, depth):
    """Grouped-lane (Q = 2, 4), one-lane (Q = 1; 2 or 4 steps in flight) and producer/consumer
    (4 consumers per block) sweeps; the latter two are chained only on request (FREI_CHAIN=2)."""
    lam, p, T0, tabs = _case(fa, nL)
    eng = fa.Engine(lam, p, tabs)
    out = {}
    try:
        eng.set_option("group_q", q)
        eng.set_option("group_waves", waves)
        if depth == "pipe":
            eng.set_option("pipe", 4)
        elif depth:
            eng.set_option("prefetch_depth", depth)
        launched = {}
        for chain in (2 if q == 1 else 1, 0):   # one-lane and pipe: chained on request
            eng.set_option("chain", chain)
            n0 = eng.chain_count()
            out[chain] = _exercise(eng, T0, nL, lam.size)
            launched[chain] = eng.chain_count() - n0
        path = eng.path()
    finally:
        eng.close()
    assert path["contracted"] and (path["paired"], path["quad"]) == (q == 2, q == 4)
    assert (path["pipe"] == 4) == (depth == "pipe")
    on = max(out)
    # the chain-on runs really chained (else the comparison below is vacuous), the others never
    assert launched[on] > 0 and launched[0] == 0, launched
    _compare(out[on], out[0], f"Q{q} waves {waves} depth {depth} nL {nL}")
    assert 1 < out[on]["run"]["n_iter"] <= 80


def test_chained_launches_with_p2p_exchange(fa):
    """The deferred update pushes and waits on the P2P mailboxes from inside the chained launch."""
    from frei_amd.distributed import p2p_comm
    from frei_amd.rendezvous import Rendezvous
    nL = 30
    lam, p, T0, tabs = _case(fa, nL)
    out = {}
    for chain in (1, 0):
        eng = fa.Engine(lam, p, tabs, comm=p2p_comm(Rendezvous(1, 0)))
        try:
            eng.set_option("group_q", 2)
            eng.set_option("group_waves", 8)
            eng.set_option("chain", chain)
            out[chain] = _exercise(eng, T0, nL, lam.size)
            out[chain]["chained"] = eng.chain_count()
        finally:
            eng.close()
    assert out[1]["chained"] > 0 and out[0]["chained"] == 0
    _compare(out[1], out[0], "p2p")


def test_no_chained_launch_while_timing(fa):
    """Per-sweep HIP events time the sweep alone: with timing on, sweep and update launch
    separately (a chained launch would also hold the deferred update and its P2P wait)."""
    nL = 30
    lam, p, T0, tabs = _case(fa, nL)
    eng = fa.Engine(lam, p, tabs)
    try:
        eng.set_option("group_q", 2)
        eng.set_option("chain", 1)
        eng.state_init(T0)
        eng.iterate(3)
        eng.synchronize()
        n0 = eng.chain_count()
        assert n0 > 0
        eng.timing(True)
        eng.iterate(3)
        eng.synchronize()
        ms, n = eng.timing_read()
        eng.timing(False)
        assert eng.chain_count() == n0 and n == 6 and ms > 0
    finally:
        eng.close()
