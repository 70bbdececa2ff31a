"""Full-size (C3: 60 layers x 500k lambda x 8 species) properties on the GPU.

The oracle cannot run 500k wavelengths in test time, so at BASELINE.json's full size the
checks are size-independent properties of the path:
- determinism: two runs give bitwise identical temperatures, spectra and dtaus;
- the default sweep at this size (two wavelengths per lane, `lam2`) against the one-lane sweep:
  temperatures within 1e-12 (only the bolometric summation tree differs);
- the grouped-lane sweep (2 lanes per wavelength, forced) against the one-lane sweep:
  temperatures within 1e-12 (likewise);
- the producer/consumer sweep (four consumers per block, forced at this size) against the
  one-lane sweep: bitwise identical temperatures, spectra and dtaus;
- the species contraction (K3) against the per-species sum in the sweep: within the
  parity tolerance (the species sum is reordered);
- physical sanity: finite, positive fluxes and a spectrum that responds to T.
"""
import numpy as np
import pytest

from tests.parity import rel

pytestmark = pytest.mark.gpu


def _engine(monkeypatch, env):
    import frei_amd as fa
    from frei_amd.workloads import c3
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    w = c3()
    tabs = {n: fa.SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, n in enumerate(w["names"])}
    eng = fa.Engine(w["lam"], w["p"], tabs, mmr=w["mmr"])
    for k in env:
        monkeypatch.delenv(k)
    return eng, w


def _run(eng, w, n=6):
    out = eng.run(w["T0"], n_timesteps=n, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
    return out


def test_full_size_properties(monkeypatch):
    runs = {}
    variants = (("default", {}), ("again", {}), ("one_lane", {"FREI_LAM2": "0"}),
                ("pair", {"FREI_GROUP_Q": "2", "FREI_SHARED_MAX_BLOCKS": "100000"}),
                ("pipe", {"FREI_PIPE": "4", "FREI_SHARED_MAX_BLOCKS": "100000"}),
                ("per_species", {"FREI_PRECONTRACT": "0"}))
    for name, env in variants:
        eng, w = _engine(monkeypatch, env)
        try:
            path = eng.path()
            if name == "pair":
                assert path["paired"]
            if name == "default":
                assert path["lam2"]
            if name == "one_lane":
                assert not path["lam2"] and not path["paired"] and path["pipe"] == 0
            if name == "pipe":
                assert path["pipe"] == 4
            if name == "per_species":
                assert not path["contracted"]
            else:
                assert path["contracted"]
            runs[name] = _run(eng, w)
        finally:
            eng.close()
    a, b = runs["default"], runs["again"]
    assert np.array_equal(a["final_T"], b["final_T"])
    assert np.array_equal(a["spectrum"], b["spectrum"])
    assert np.array_equal(a["dtaus"], b["dtaus"])
    assert np.isfinite(a["spectrum"]).all() and (a["spectrum"] > 0).all()
    assert np.isfinite(a["dtaus"]).all()
    one = runs["one_lane"]
    for k in ("final_T", "spectrum", "dtaus"):
        assert np.array_equal(runs["pipe"][k], one[k]), k
    for v in ("default", "pair"):
        assert rel(runs[v]["final_T"], one["final_T"]) < 1e-12, v
        assert rel(runs[v]["spectrum"], one["spectrum"]) < 1e-9, v
    assert rel(runs["per_species"]["final_T"], a["final_T"]) < 1e-10
    # the T-P loop moved the temperatures (6 iterations from the initial profile)
    assert rel(a["final_T"], w_T0()) > 1e-6


def w_T0():
    from frei_amd.workloads import c3
    return c3(n_lam=1000)["T0"]
