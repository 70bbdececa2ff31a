"""Trailing update (option ``tail``, FREI_TAIL, round 6): the producer/consumer sweep's launch
carries its own fused update as trailing workgroups, which reduce each layer as soon as every
sweep block has published that layer's steps (frei_kernels.hip sweep_pipe_tail_kernel) instead of
in a separate kernel after the sweep.  The reduction tree and the update's expressions are the
separate update kernel's, so every output must be bit-identical to tail = 0: single sweeps,
fixed-count iterations and runs to convergence, odd and even layer counts, one and two phases of
table rows in flight, with the one-rank P2P exchange inside the trailing update, and the C4
8-GPU slice (60 x 62.5k lambda x 8 species) run to radiative equilibrium."""
import numpy as np
import pytest

from tests.test_gpu_chain import _case, _compare, _exercise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fa():
    import frei_amd
    return frei_amd


def _both(eng, T0, nL, n_lam):
    out, launched = {}, {}
    for tail in (1, 0):
        eng.set_option("tail", tail)
        n0 = eng.tail_count()
        out[tail] = _exercise(eng, T0, nL, n_lam)
        launched[tail] = eng.tail_count() - n0
    # the tail-on runs really ran trailing updates (else the comparison is vacuous), the others not
    assert launched[1] > 0 and launched[0] == 0, launched
    return out


@pytest.mark.parametrize("nL", [30, 31, 60])
@pytest.mark.parametrize("pf", [1, 2])
def test_trailing_update_is_bitwise_identical(fa, nL, pf):
    lam, p, T0, tabs = _case(fa, nL)
    eng = fa.Engine(lam, p, tabs)
    try:
        eng.set_option("pipe", 4)
        eng.set_option("pipe_pf", pf)
        path = eng.path()
        out = _both(eng, T0, nL, lam.size)
    finally:
        eng.close()
    assert path["pipe"] == 4 and path["tail"], path
    _compare(out[1], out[0], f"tail nL {nL} pf {pf}")
    assert 1 < out[1]["run"]["n_iter"] <= 80


def test_trailing_update_with_p2p_exchange(fa):
    """The trailing update pushes and waits on the P2P mailboxes from inside the sweep's launch."""
    from frei_amd.distributed import p2p_comm
    from frei_amd.rendezvous import Rendezvous
    nL = 30
    lam, p, T0, tabs = _case(fa, nL)
    out = {}
    for tail in (1, 0):
        eng = fa.Engine(lam, p, tabs, comm=p2p_comm(Rendezvous(1, 0)))
        try:
            eng.set_option("pipe", 4)
            eng.set_option("tail", tail)
            out[tail] = _exercise(eng, T0, nL, lam.size)
            out[tail]["launched"] = eng.tail_count()
        finally:
            eng.close()
    assert out[1]["launched"] > 0 and out[0]["launched"] == 0
    _compare(out[1], out[0], "tail p2p")


def test_no_trailing_update_while_timing(fa):
    """Per-sweep HIP events time the sweep alone: with timing on, sweep and update launch
    separately."""
    nL = 30
    lam, p, T0, tabs = _case(fa, nL)
    eng = fa.Engine(lam, p, tabs)
    try:
        eng.set_option("pipe", 4)
        eng.state_init(T0)
        eng.iterate(3)
        eng.synchronize()
        n0 = eng.tail_count()
        assert n0 == 6
        eng.timing(True)
        eng.iterate(3)
        eng.synchronize()
        ms, n = eng.timing_read()
        eng.timing(False)
        assert eng.tail_count() == n0 and n == 6 and ms > 0
        eng.iterate(2)
        eng.synchronize()
        assert eng.tail_count() == n0 + 4
    finally:
        eng.close()


def test_trailing_update_c4_slice_radiative_equilibrium(fa):
    """The 8-GPU slice the trailing update is for: C3's 60 layers x 8 species on 62,500
    wavelengths (245 producer/consumer blocks, the update in four trailing blocks), run to the
    reference's radiative equilibrium and for fixed iterations — bitwise tail = 0."""
    from frei_amd.engine import Engine
    from frei_amd.opacity import SeparableTable
    from frei_amd.workloads import c3
    w = c3(n_layers=60, n_lam=500_000, n_T=16)
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, n in enumerate(w["names"])}
    eng = Engine(w["lam"], w["p"], tabs, mmr=w["mmr"], lam_slice=(0, 62_500))
    out = {}
    try:
        path = eng.path()
        for tail in (1, 0):
            eng.set_option("tail", tail)
            r = eng.run(w["T0"], n_timesteps=200, n_zero_crossings=2, convergence_dT=3.0,
                        alpha=1.0)
            eng.state_init(w["T0"])
            eng.iterate(9, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
            eng.synchronize()
            out[tail] = (r, eng.get_temperatures(), eng.get_fluxes(), eng.tail_count())
    finally:
        eng.close()
    assert path["pipe"] == 4 and path["tail"], path
    r1, r0 = out[1][0], out[0][0]
    assert out[1][3] > 0 and out[0][3] == out[1][3]    # tail = 0 added no trailing launches
    assert r1["n_iter"] == r0["n_iter"] and 1 < r1["n_iter"] < 200
    for k in ("final_T", "temp_hist", "spectrum", "dtaus"):
        assert np.array_equal(r1[k], r0[k]), k
    assert np.array_equal(out[1][1], out[0][1])
    for i in (0, 1):
        assert np.array_equal(out[1][2][i], out[0][2][i])
