"""Host-side logic that needs no GPU: cross-section file readers, binned_opacity's species
selection, the batched API's argument checks, and the benchmark's byte accounting (which
must select the same source rows as the binning plan the oracle pins)."""
import os

import numpy as np
import pytest

from oracle import frei_oracle as O


def _xsec_arrays():
    wl = np.linspace(0.5, 10.0, 40)
    T = np.array([1000.0, 2000.0])
    p = np.array([1e-3, 1.0, 10.0])
    op = np.arange(2 * 3 * 40, dtype=np.float32).reshape(2, 3, 40)
    return op, T, p, wl


def test_open_cross_section_npz_and_netcdf3(tmp_path):
    import frei_amd as fa
    op, T, p, wl = _xsec_arrays()
    path = tmp_path / "1H2-16O_test.npz"
    np.savez(path, opacity=op, temperature=T, pressure=p, wavelength=wl)
    x = fa.open_cross_section(str(path))
    assert x.isotopologue == "1H2-16O" and x.opacity.dtype == np.float32
    assert np.array_equal(x.opacity, op) and np.array_equal(x.wavelength, wl)
    from scipy.io import netcdf_file
    nc = tmp_path / "12C-16O_test.nc"
    with netcdf_file(str(nc), "w") as f:
        f.createDimension("temperature", 2)
        f.createDimension("pressure", 3)
        f.createDimension("wavelength", 40)
        for name, dims, arr in (("temperature", ("temperature",), T),
                                ("pressure", ("pressure",), p),
                                ("wavelength", ("wavelength",), wl),
                                ("opacity", ("temperature", "pressure", "wavelength"), op)):
            v = f.createVariable(name, arr.dtype, dims)
            v[:] = arr
    y = fa.open_cross_section(str(nc))
    assert y.isotopologue == "12C-16O"
    assert np.array_equal(y.opacity, op) and np.array_equal(y.pressure, p)
    hdf = tmp_path / "1H2-16O_hdf.nc"
    hdf.write_bytes(b"\x89HDF\r\n\x1a\n" + b"\0" * 16)
    with pytest.raises(ValueError, match="netCDF4/HDF5"):
        fa.open_cross_section(str(hdf))


def test_binned_opacity_selects_species_from_files(tmp_path):
    import frei_amd as fa
    op, T, p, wl = _xsec_arrays()
    for iso in ("1H2-16O", "12C-16O", "Na"):
        np.savez(tmp_path / f"{iso}_x.npz", opacity=op, temperature=T, pressure=p,
                 wavelength=wl)
    lam, wl_bins, _ = O.wavelength_grid(0.6, 9.0, 10)
    T_t, p_t = np.array([1500.0, 1800.0]), np.array([5.0, 0.1])
    tabs = fa.binned_opacity(T_t, p_t, wl_bins, lam, species=["H2O", "Na"],
                             path=str(tmp_path / "*.nc"))
    assert sorted(tabs) == ["1H2-16O", "Na"]
    t = tabs["Na"]
    assert t.shape == (2, 2, 10) and t.groupies and np.array_equal(t.pressure, p_t)
    with pytest.raises(FileNotFoundError):
        fa.binned_opacity(T_t, p_t, wl_bins, lam, path=str(tmp_path / "none_*.nc"))


def test_batched_grids_must_share_grids_and_tables():
    import frei_amd as fa
    pl = fa.Planet.from_hot_jupiter()
    a = fa.Grid(pl, n_wl_bins=64, n_layers=8)
    b = fa.Grid(pl, n_wl_bins=65, n_layers=8)
    a.load_opacities(opacities=fa.load_example_opacity(a))
    b.load_opacities(opacities=a.opacities)
    with pytest.raises(ValueError, match="wavelengths and pressures"):
        fa.batched_emission_spectra([a, b])
    c = fa.Grid(pl, n_wl_bins=64, n_layers=8)
    c.load_opacities(opacities=fa.load_example_opacity(c))
    with pytest.raises(ValueError, match="one opacity dict"):
        fa.batched_emission_spectra([a, c])


def test_binning_accounting_selects_the_oracle_rows():
    from frei_amd.workloads import binning_bytes, binning_workload, nearest_index
    w = binning_workload(n_layers=12, n_lam=2000, spacing_cm=2.0, n_T_src=7, n_p_src=5)
    assert np.array_equal(nearest_index(w["T_src"], w["T0"]), O.nearest_index(w["T_src"], w["T0"]))
    assert np.array_equal(nearest_index(w["p_src"], w["p"]), O.nearest_index(w["p_src"], w["p"]))
    acc = binning_bytes(w)
    start, end = O.bin_ranges(w["wl_hi"], w["wl_bins"])
    assert acc["points"] == int(end[-1] - start[0])
    rows = {(t, q) for t in O.nearest_index(w["T_src"], w["T0"])
            for q in O.nearest_index(w["p_src"], w["p"])}
    assert acc["source_rows"] == len(rows) and acc["dest_rows"] == 144


def test_build_script_lists_every_hip_source():
    from frei_amd import build
    here = os.path.join(os.path.dirname(build.__file__), "csrc")
    hips = sorted(f for f in os.listdir(here) if f.endswith(".hip"))
    assert sorted(os.path.basename(s) for s in build.SOURCES) == hips


def test_chemistry_table_interpolation_contract():
    """The ChemistryTable interface (engine: frei_set_chemistry; checker:
    oracle.ChemistryTable): exact at nodes, linear in T and log10 p between them, clamped
    outside; the host wrapper orders species like the opacity dict."""
    import numpy as np
    import frei_amd as fa
    from oracle import frei_oracle as O
    T = np.array([500.0, 1000.0, 2000.0])
    p = np.array([1e-4, 1e-2, 1.0, 100.0])
    vals = np.arange(2 * 3 * 4, dtype=float).reshape(2, 3, 4) + 1.0
    c = O.ChemistryTable(vals, T, p)
    for i, t in enumerate(T):
        for j, pb in enumerate(p):
            assert np.allclose(c(t, pb), vals[:, i, j], rtol=1e-14, atol=0)
    mid = c(750.0, 1e-3)     # halfway in T and in log10 p
    assert np.allclose(mid, vals[:, :2, :2].mean(axis=(1, 2)), rtol=1e-12)
    assert np.array_equal(c(10.0, 1e-9), vals[:, 0, 0])      # clamped below
    assert np.array_equal(c(9e3, 1e5), vals[:, -1, -1])     # clamped above
    t = fa.ChemistryTable({"12C-16O": vals[1], "1H2-16O": vals[0]}, T, p)
    assert np.array_equal(t.array(["1H2-16O", "12C-16O"]), vals)


def test_balanced_edges_split_the_measured_cost_evenly():
    """Cost-balanced wavelength slices (bench.py's multi-GPU calibration): equal costs keep an
    even split, a slice twice as expensive per wavelength is shrunk, edges stay block-aligned."""
    from frei_amd.engine import balanced_edges, partition
    n, R = 500_000, 8
    even = [partition(n, R, r)[0] for r in range(R)] + [n]
    e = balanced_edges(even, [1.0] * R)
    assert e[0] == 0 and e[-1] == n and all(b > a for a, b in zip(e, e[1:]))
    assert max(abs(a - b) for a, b in zip(e, even)) <= 256
    assert all(x % 256 == 0 for x in e[:-1])
    # the last slice costs twice as much per wavelength: the new split equalises the cost
    costs = [1.0] * (R - 1) + [2.0]
    e = balanced_edges(even, costs)
    dens = np.repeat(np.array(costs) / np.diff(even), np.diff(even))
    per = [dens[a:b].sum() for a, b in zip(e, e[1:])]
    assert max(per) / min(per) < 1.01
    assert e[-1] - e[-2] < n // R
    with pytest.raises(ValueError):
        balanced_edges([0, 10, 5], [1.0, 1.0])


def test_chemistry_provider_called_on_the_reference_signature():
    """frei_amd.chemistry.provider_mmr calls a provider as the reference's kappa does
    (chemistry(T, p, species, m_bar=...), opacity.py:246-248) and reads its dict; the reference's
    mock as a provider is detected as T-independent, a T-dependent one is not; a species the
    provider does not return raises."""
    import numpy as np
    import importlib
    C = importlib.import_module("frei_amd.chemistry")   # the package re-exports the function
    names = ["1H2-16O", "12C-16O"]
    p = np.array([10.0, 1.0, 0.1])
    seen = []

    def fake(T, pr, species, return_vmr=False, m_bar=None):
        seen.append((np.asarray(T).shape, list(species), m_bar))
        T = np.asarray(getattr(T, "value", T), dtype=float)
        return {"1H2-16O": 1e-3 * (T / 1000.0), "12C-16O": np.full(T.shape, 2e-3)}
    v = C.provider_mmr(fake, [1000.0, 2000.0], [1.0, 0.1], names, 4e-24)
    assert np.allclose(v, [[1e-3, 2e-3], [2e-3, 2e-3]])
    assert seen[0][1] == names and float(getattr(seen[0][2], "value", seen[0][2])) == 4e-24
    assert C.fixed_provider_mmr(fake, names, p, 4e-24) is None
    fixed = C.fixed_provider_mmr(C.chemistry, names, p, 4e-24)
    mock = C.chemistry(np.full(3, 1000.0), p, names, m_bar=4e-24)
    assert np.array_equal(fixed, np.array([mock[n] for n in names]))
    import pytest
    with pytest.raises(KeyError, match="12C-1H4"):
        C.provider_mmr(fake, [1000.0], [1.0], names + ["12C-1H4"], 4e-24)


def test_every_floor_family_names_an_existing_outright_twin():
    """tests/parity.py OUTRIGHT_TWINS: each floor-rule test family names a well-conditioned twin
    held to 1e-10 outright; the twin's test function (and the parameter id, where one is named)
    exists in the tree."""
    import ast
    import pathlib
    import re
    from tests.parity import OUTRIGHT_TWINS
    root = pathlib.Path(__file__).resolve().parents[1]
    for family, twin in OUTRIGHT_TWINS.items():
        path, node = twin.split("::")
        src = (root / path).read_text()
        fn = node.split("[")[0]
        funcs = {n.name for n in ast.walk(ast.parse(src)) if isinstance(n, ast.FunctionDef)}
        assert fn in funcs, twin
        assert re.search(rf"def {family}\(", (root / "tests").joinpath(
            next(p.name for p in (root / "tests").glob("test_gpu_*.py")
                 if f"def {family}(" in p.read_text())).read_text()), family
