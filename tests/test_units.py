"""Quantity handling at the Python seam (frei_amd/units.py), on CPU: a caller-owned Quantity
is written in place through its own unit, plain arrays stay plain, and results carry the
reference's units when the caller passed Quantities (twostream.py:334-339, 418-421;
opacity.py:269).  The stand-in (tests/quantity.py) refuses unitless assignment as astropy
does."""
import numpy as np
import pytest

from frei_amd.units import assign, unit_of, value, with_unit
from tests.quantity import Quantity, Unit, UnitConversionError, q


def test_standin_refuses_unitless_assignment_like_astropy():
    f = q(np.zeros((3, 4)), "erg / (s cm3)")
    with pytest.raises(UnitConversionError):
        f[...] = np.ones((3, 4))
    f[1] = q(np.ones(4), "erg / (s cm3)")
    assert isinstance(f, np.ndarray) and f.dtype == np.float64
    assert np.array_equal(f.value[1], np.ones(4))


def test_assign_writes_quantities_in_place_through_their_unit():
    rng = np.random.default_rng(0)
    src = rng.random((5, 7))
    f = q(np.zeros((5, 7)), "erg / (s cm3)")
    out = assign(f, src, "erg / (s cm3)")
    assert out is f and isinstance(out, Quantity)
    assert np.array_equal(f.value, src)                 # same unit: bit for bit
    w = q(np.zeros((5, 7)), "W / m3")                   # another unit: converted
    assign(w, src, "erg / (s cm3)")
    assert np.allclose(w.value, src * 0.1, rtol=1e-15)
    plain = np.zeros((5, 7))
    assert assign(plain, src, "erg / (s cm3)") is plain and np.array_equal(plain, src)
    assert assign(None, src, "erg / (s cm3)") is src


def test_unit_of_and_with_unit():
    T = q([1000.0, 1200.0], "K")
    lam = q([1.0, 2.0], "um")
    assert unit_of("K", None, lam, T) == Unit("K")       # first Quantity that converts
    assert unit_of("K", np.ones(2), 3.0) is None         # no Quantity in: plain out
    x = with_unit(np.arange(3.0), Unit("K"))
    assert isinstance(x, Quantity) and x.unit == Unit("K")
    assert with_unit(np.arange(3.0), None).__class__ is np.ndarray
    assert np.array_equal(value(q([1.0, 2.0], "um"), "cm"), [1e-4, 2e-4])
