"""A minimal stand-in for astropy's ``Quantity`` (the GPU box has no astropy), with the two
behaviours the reference's emit/absorb seam relies on (twostream.py:334-339, 392-394;
core.py:265-299):

- it is an ``ndarray`` subclass carrying ``.unit`` with ``.to(unit)`` / ``.value``, so
  ``isinstance(q, np.ndarray)`` and ``q.dtype == float64`` hold, as they do for astropy;
- ``q[...] = x`` refuses a unitless ``x`` (astropy: ``UnitConversionError: '' (dimensionless)
  and 'erg / (cm3 s)' are not convertible``) and converts a Quantity ``x`` to ``q``'s unit.

Units are (dimension, scale-to-cgs) pairs over the handful the seam uses.  Test
infrastructure only."""
import numpy as np


class UnitConversionError(ValueError):
    pass


_UNITS = {
    "K": ("temperature", 1.0),
    "bar": ("pressure", 1e6),
    "dyn / cm2": ("pressure", 1.0),
    "um": ("length", 1e-4),
    "cm": ("length", 1.0),
    "g": ("mass", 1.0),
    "cm / s2": ("acceleration", 1.0),
    "erg / (s cm3)": ("flux density", 1.0),
    "W / m3": ("flux density", 1e7 / 1e6),
}


class Unit:
    __array_ufunc__ = None              # ndarray * unit defers to Unit.__rmul__, as in astropy

    def __init__(self, name):
        if name not in _UNITS:
            raise ValueError(f"stand-in unit {name!r} unknown")
        self.name = name
        self.dim, self.scale = _UNITS[name]

    def __rmul__(self, other):          # array * unit -> Quantity (astropy's idiom)
        return Quantity(other, self)

    def factor_to(self, other):
        if self.dim != other.dim:
            raise UnitConversionError(f"'{self.name}' and '{other.name}' are not convertible")
        return self.scale / other.scale

    def __eq__(self, other):
        return isinstance(other, Unit) and other.name == self.name

    def __hash__(self):
        return hash(self.name)

    def __repr__(self):
        return f"Unit({self.name!r})"


def _unit(u):
    return u if isinstance(u, Unit) else Unit(u)


class Quantity(np.ndarray):
    def __new__(cls, values, unit):
        obj = np.array(values, dtype=float).view(cls)
        obj.unit = _unit(unit)
        return obj

    def __array_finalize__(self, obj):
        self.unit = getattr(obj, "unit", None)

    @property
    def value(self):
        return self.view(np.ndarray)

    def to(self, unit):
        u = _unit(unit)
        f = self.unit.factor_to(u)
        return Quantity(self.view(np.ndarray) if f == 1.0 else self.view(np.ndarray) * f, u)

    def __setitem__(self, key, val):
        if not isinstance(val, Quantity):
            raise UnitConversionError(
                f"'' (dimensionless) and '{self.unit.name}' are not convertible")
        np.ndarray.__setitem__(self.view(np.ndarray), key, val.to(self.unit).view(np.ndarray))


def q(values, unit):
    return Quantity(values, unit)
