"""Host side of the drop-in boundary for opacity tables: the reference's DataArrays are
addressed by dimension NAME (opacity.py:252-263) and come in three layouts (load_example_opacity
(p, T, λ); binned_opacity groupies (T, p, λ), interp.py:287-307; binned_opacity exact, the
Grid.load_opacities default, (λ, T, p), opacity.py:42, 156-167).  frei_amd.opacity.table_values
must hand the engine (p, T, λ) for every one of them — no GPU needed for this part."""
import numpy as np
import pytest

from tests.dataarray import DataArrayLike, reference_layouts


def test_table_values_transposes_every_reference_layout_by_name():
    from frei_amd.opacity import table_values
    rng = np.random.default_rng(0)
    n = 5                                       # n_T = n_p, as on every Grid
    v = rng.random((n, n, 11))
    lay = reference_layouts(v, np.geomspace(100, 1e-4, n), np.linspace(2000, 900, n),
                            np.linspace(1, 2, 11))
    for name, da in lay.items():
        out = table_values(da)
        assert out.shape == v.shape and np.array_equal(out, v), name


def test_table_values_on_reference_binned_goldens(golden):
    """The reference's own binned tables in the layouts make_binning_goldens.py asserted on
    its output."""
    from frei_amd.opacity import table_values
    B = golden("binning.npz")
    gro = DataArrayLike(B["g1_groupies"], ("temperature", "pressure", "wavelength"),
                        temperature=B["g1_T"], pressure=B["g1_p"], wavelength=B["g1_lam"])
    exa = DataArrayLike(B["g1_exact"], ("wavelength", "temperature", "pressure"),
                        temperature=B["g1_T"], pressure=B["g1_p"], wavelength=B["g1_lam"])
    a, b = table_values(gro), table_values(exa)
    assert a.shape == b.shape == (B["g1_p"].size, B["g1_T"].size, B["g1_lam"].size)
    # value at (p index 1, T index 4, λ 17) picked by name from the raw arrays
    assert a[1, 4, 17] == B["g1_groupies"][4, 1, 17]
    assert b[1, 4, 17] == B["g1_exact"][17, 4, 1]
    # n_T = n_p here: a positional read of the groupies table would be a silent transpose
    assert B["g1_T"].size == B["g1_p"].size
    assert not np.array_equal(a, B["g1_groupies"])


def test_tables_without_dims_keep_the_positional_layout():
    from frei_amd.opacity import OpacityTable, table_values

    class Plain:
        values = np.arange(24.0).reshape(2, 3, 4)
    assert np.array_equal(table_values(Plain()), Plain.values)
    t = OpacityTable(Plain.values, [1.0, 0.1], [1000.0, 1500.0, 2000.0])
    assert np.array_equal(table_values(t), Plain.values)


def test_opacity_table_takes_dims_and_dataarrays():
    from frei_amd.opacity import OpacityTable
    v = np.arange(2 * 3 * 4, dtype=float).reshape(2, 3, 4)   # (p, T, λ)
    p, T, lam = [1.0, 0.1], [1000.0, 1500.0, 2000.0], [1.0, 2.0, 3.0, 4.0]
    t = OpacityTable(np.transpose(v, (2, 1, 0)), p, T, dims=("wavelength", "temperature",
                                                              "pressure"))
    assert np.array_equal(t.values, v)
    for da in reference_layouts(v, p, T, lam).values():
        u = OpacityTable.from_dataarray(da)
        assert np.array_equal(u.values, v) and np.array_equal(u.wavelength, lam)


def test_unknown_dims_raise_instead_of_guessing():
    from frei_amd.opacity import table_values
    bad = DataArrayLike(np.zeros((2, 2, 3)), ("temperature", "pressure", "wavenumber"))
    with pytest.raises(ValueError, match="permutation"):
        table_values(bad)
    two = DataArrayLike(np.zeros((2, 3)), ("pressure", "wavelength"))
    with pytest.raises(ValueError, match="permutation"):
        table_values(two)
