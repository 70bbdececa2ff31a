"""The fused reduce + update launch (one workgroup per layer, frei_kernels.hip
update_fused_kernel) against the two-kernel form (reduce_kernel + update_kernel,
``fused_update`` 0): same summation order for the partial sums, same dT expression, same
bookkeeping, so single sweeps and whole T-P runs must agree bit for bit — on every sweep path
the tables can select (contracted one-lane and grouped-lane, per-species, per-species
brackets, generic, T-dependent chemistry, a 400-layer atmosphere)."""
import numpy as np
import pytest

import oracle.frei_oracle as O

pytestmark = pytest.mark.gpu

M_BAR = 2.4 * 1.6605390666e-24


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    return frei_amd


def _case(fa, name):
    rng = np.random.default_rng(57)
    nL, n_lam = (400, 700) if name == "deep" else (30, 5000)
    lam, _, _ = O.wavelength_grid(0.5, 10, n_lam)
    p = O.pressure_grid(nL, -6, np.log10(200))
    T0 = O.temperature_grid(p, 2200.0, 0.1, 0.1)
    names = ["1H2-16O", "12C-16O", "12C-1H4"]
    pn = np.logspace(np.log10(300), -7, 11) if name == "offnode_p" else p
    Tns = [np.linspace(0.7 * T0.min(), 1.3 * T0.max(), 9)] * 3
    if name == "mixed_T":
        Tns = [np.linspace(0.6 * T0.min(), 1.4 * T0.max(), 7 + 2 * s) for s in range(3)]
    tabs = {n: fa.SeparableTable(10 ** rng.uniform(-3, 1, lam.size), (pn / 1.0) ** 0.1,
                                 (Tn / 1000.0) ** 0.5, pn, Tn) for n, Tn in zip(names, Tns)}
    mmr = None
    if name == "chemistry":
        cT = np.linspace(300.0, 4000.0, 12)
        cp = np.logspace(-7, 3, 8)
        x = np.tanh((cT[:, None] - 1500.0) / 400.0) + 0.05 * np.log10(cp)[None, :]
        base = O.mock_mmr(names, M_BAR)
        mmr = fa.ChemistryTable({n: base[s] * 10 ** (0.8 * (-1) ** s * x)
                                 for s, n in enumerate(names)}, cT, cp)
    return lam, p, T0, tabs, mmr


def _exercise(eng, T0, nL, n_lam):
    rng = np.random.default_rng(3)
    up0 = 10 ** rng.uniform(8, 12, (nL, n_lam))
    dn0 = 10 ** rng.uniform(6, 11, (nL, n_lam))
    r = {}
    for d in (0, 1):
        eng.set_temperatures(T0)
        eng.set_fluxes(up0, dn0)
        r[d] = eng.sweep(d, alpha=1.0) + eng.get_fluxes() + (eng.get_temperatures(),)
    r["run"] = eng.run(T0, n_timesteps=80)
    r["run2"] = eng.run(T0, n_timesteps=5, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
    eng.state_init(T0)
    eng.iterate(7, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
    eng.synchronize()
    r["iterate"] = eng.get_temperatures()
    return r


def _same(a, b, what):
    assert np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True), what


@pytest.mark.parametrize("name,opts", [
    ("contracted", {}),
    ("contracted", {"group_q": 1}),
    ("contracted", {"group_q": 2}),
    ("contracted", {"group_q": 1, "shared": 0, "lam2": 1}),   # two wavelengths per lane
    ("per_species", {"precontract": 0}),
    ("mixed_T", {}),
    ("offnode_p", {}),
    ("chemistry", {}),
    ("deep", {}),
])
def test_fused_update_is_bitwise_identical_to_two_kernels(fa, name, opts):
    lam, p, T0, tabs, mmr = _case(fa, name)
    eng = fa.Engine(lam, p, tabs, mmr=mmr)
    out = {}
    try:
        for k, v in opts.items():
            eng.set_option(k, v)
        for fused in (1, 0):
            eng.set_option("fused_update", fused)
            out[fused] = _exercise(eng, T0, p.size, lam.size)
        path = eng.path()
    finally:
        eng.close()
    if name == "contracted":
        assert path["contracted"]
        assert path["lam2"] == bool(opts.get("lam2", 0))
    if name in ("per_species", "chemistry"):
        assert not path["contracted"]
    a, b = out[1], out[0]
    for d in (0, 1):
        for i, what in enumerate(("dT", "bolometric", "dtaus", "F_up", "F_down", "T")):
            _same(a[d][i], b[d][i], f"{name} dir {d} {what}")
    for key in ("run", "run2"):
        assert a[key]["n_iter"] == b[key]["n_iter"]
        for what in ("final_T", "temp_hist", "spectrum", "dtaus"):
            _same(a[key][what], b[key][what], f"{name} {key} {what}")
    _same(a["iterate"], b["iterate"], f"{name} iterate T")
    assert 1 < a["run"]["n_iter"] <= 80


@pytest.mark.parametrize("name,opts", [("contracted", {}), ("per_species", {"precontract": 0}),
                                       ("contracted", {"group_q": 2}),
                                       ("contracted", {"group_q": 1, "shared": 0, "lam2": 1})])
def test_graph_replay_is_bitwise_identical_to_launches(fa, name, opts):
    """T-P iterations replayed from a captured hipGraph (frei_iterate / frei_run) against
    kernel-by-kernel launches: same kernels, same arguments, so bit-identical state; the graph
    is captured once and reused while the arguments repeat."""
    lam, p, T0, tabs, mmr = _case(fa, name)
    eng = fa.Engine(lam, p, tabs, mmr=mmr)
    out = {}
    try:
        for k, v in opts.items():
            eng.set_option(k, v)
        for graph in (1, 0):
            eng.set_option("graph", graph)
            r = {}
            r["run"] = eng.run(T0, n_timesteps=80)
            r["run_again"] = eng.run(T0, n_timesteps=80)
            eng.state_init(T0)
            eng.iterate(9, n_zero_crossings=10 ** 6, convergence_dT=-1.0)   # 2 replays + 1
            eng.synchronize()
            r["iterate"] = eng.get_temperatures()
            out[graph] = r
            if graph:
                cap, rep = eng.graph_info()
                # run's stop/threshold arguments differ from iterate's: two graphs in total
                assert cap == 2 and rep >= 4, (cap, rep)
    finally:
        eng.close()
    a, b = out[1], out[0]
    for key in ("run", "run_again"):
        assert a[key]["n_iter"] == b[key]["n_iter"]
        for what in ("final_T", "temp_hist", "spectrum", "dtaus"):
            _same(a[key][what], b[key][what], f"{name} {key} {what}")
    _same(a["run"]["final_T"], a["run_again"]["final_T"], "graph reuse")
    _same(a["iterate"], b["iterate"], f"{name} iterate T")


def test_graph_key_pass_keeps_record_state_when_rec_sweep_changes(fa):
    """The graph key pass (a dry iteration that only hashes launch arguments) must not clear the
    'last update wrote no step records' flag: with records formed in the sweep, then turned off
    between two frei_iterate calls, the first real sweep must write its own records first — the
    graph path gives bitwise the direct path's temperatures."""
    lam, p, T0, tabs, mmr = _case(fa, "contracted")
    out = {}
    for graph in (1, 0):
        eng = fa.Engine(lam, p, tabs, mmr=mmr)
        try:
            eng.set_option("graph", graph)
            eng.set_option("rec_sweep", 1)
            eng.state_init(T0)
            eng.iterate(5, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            eng.set_option("rec_sweep", 0)
            eng.iterate(5, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            eng.synchronize()
            out[graph] = eng.get_temperatures()
            if graph:
                cap, rep = eng.graph_info()
                assert cap >= 1 and rep >= 1, (cap, rep)
        finally:
            eng.close()
    _same(out[1], out[0], "graph vs direct after a rec_sweep change")
