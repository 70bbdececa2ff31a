"""Unit handling without astropy.

The reference takes astropy ``Quantity`` objects everywhere.  astropy is not part of the
MI355X image, so frei_amd accepts plain numbers/arrays in the reference's default units
(µm, bar, K, g, cm s^-2, erg s^-1 cm^-3) and, when astropy IS importable, Quantities,
which are converted with ``.to(unit)``.  When the caller passed Quantities, results go back
as Quantities in the reference's units (``with_unit``), and caller-owned Quantity arrays are
written in place through their own unit (``assign``), as the reference's emit/absorb mutate
``fluxes_up``/``fluxes_down`` (twostream.py:334-339, 392-394, 418-421).
"""
import numpy as np


def is_quantity(x):
    return hasattr(x, "unit") and hasattr(x, "to")


def value(x, unit):
    """Strip units: Quantity -> its value in ``unit``; anything else -> float array."""
    if is_quantity(x):
        return np.asarray(x.to(unit).value, dtype=float)
    return np.asarray(x, dtype=float)


def scalar(x, unit):
    return float(value(x, unit))


def unit_of(unit, *likes):
    """The unit object for ``unit`` in the unit system of the first Quantity among ``likes``
    that converts to it (``q.to(unit).unit``); astropy's ``Unit(unit)`` when a Quantity was
    passed but none converts; None when no argument is a Quantity (plain arrays in, plain
    arrays out)."""
    quantities = [q for q in likes if is_quantity(q)]
    if not quantities:
        return None
    for q in quantities:
        try:
            return q.to(unit).unit
        except Exception:       # a different dimension (astropy UnitConversionError)
            continue
    try:
        from astropy import units as u
    except ImportError:
        return None
    return u.Unit(unit)


def with_unit(x, u):
    """``x`` as a Quantity of unit ``u`` (``x * u``), or ``x`` itself when ``u`` is None."""
    return x if u is None else x * u


def assign(dst, src, unit):
    """Write the float array ``src`` (in ``unit``) into the caller's array ``dst`` in place and
    return ``dst``.  A Quantity is written through its own unit (``src * unit`` converted to
    ``dst``'s unit by the Quantity itself, exact when the units agree); a float64 ndarray
    directly.  Anything else (None, lists, other dtypes) cannot be updated in place: ``src``
    itself is returned."""
    if is_quantity(dst):
        dst[...] = src * dst.to(unit).unit
        return dst
    if isinstance(dst, np.ndarray) and dst.dtype == np.float64:
        dst[...] = src
        return dst
    return src
