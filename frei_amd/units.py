"""Unit handling without astropy.

The reference takes astropy ``Quantity`` objects everywhere.  astropy is not part of the
MI355X image, so frei_amd accepts plain numbers/arrays in the reference's default units
(µm, bar, K, g, cm s^-2, erg s^-1 cm^-3) and, when astropy IS importable, Quantities,
which are converted with ``.to(unit)``.
"""
import numpy as np


def value(x, unit):
    """Strip units: Quantity -> its value in ``unit``; anything else -> float array."""
    if hasattr(x, "unit") and hasattr(x, "to"):
        return np.asarray(x.to(unit).value, dtype=float)
    return np.asarray(x, dtype=float)


def scalar(x, unit):
    return float(value(x, unit))
