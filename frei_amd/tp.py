"""Initial pressure / temperature grids (frei/tp.py:10-62)."""
import numpy as np

from .units import value

__all__ = ["pressure_grid", "temperature_grid"]


def pressure_grid(n_layers=30, P_toa=-6, P_boa=1.1):
    """Log-spaced pressures in bar from bottom (index 0) to top (tp.py:10-33).
    ``P_toa``/``P_boa`` are log10(bar) like the reference."""
    return np.logspace(P_toa, P_boa, n_layers)[::-1]


def temperature_grid(pressures, T_ref=2300.0, P_ref=0.1, alpha=0.1):
    """T = T_ref (p / P_ref)^alpha in K (tp.py:36-62); pressures in bar."""
    p = value(pressures, "bar")
    return value(T_ref, "K") * (p / value(P_ref, "bar")) ** alpha
