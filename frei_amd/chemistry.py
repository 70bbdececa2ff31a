"""Mass mixing ratios (frei/chemistry.py:114-246).

FastChem (``pyfastchem``, third-party C++, unpinned) is not part of this engine.  Where the
mixing ratios come from, in order:

- ``chemistry=provider``: the caller's chemistry function on the reference's signature
  (``frei.chemistry.chemistry`` itself in the drop-in), evaluated exactly where
  the reference's kappa evaluates it — every layer at its current (T, p), every sweep
  (opacity.py:246-248).  A provider found independent of T (the reference's own mock) fixes
  per-layer mixing ratios and the T-P loop stays on the device; a T-dependent one (FastChem)
  is evaluated on the host between sweeps (Engine.run).
- ``mmr=``: per-layer arrays, or a :class:`ChemistryTable` tabulated on (T, p) nodes that the
  device re-interpolates at each layer's current temperature every sweep (frei_set_chemistry).
- neither: the reference's mock (chemistry.py:142-153, 207-246): VMR = 1.5e-3 for every
  species (chemistry.py:243), mmr = VMR * mass / m_bar.
"""
import re

import numpy as np

from .constants import AMU, M_BAR_DEFAULT
from .units import value

__all__ = ["chemistry", "iso_to_species", "iso_to_mass", "ChemistryTable", "provider_mmr",
           "fixed_provider_mmr"]

MOCK_VMR = 1.5e-3

# periodictable masses of bare atoms (chemistry.py:37 falls back to periodictable)
ATOM_MASS = dict(H=1.00794, He=4.002602, C=12.0107, N=14.0067, O=15.9994, F=18.9984032,
                 Na=22.98977, Al=26.981538, Cl=35.453, K=39.0983, Ti=47.867, V=50.9415,
                 Cr=51.9961, Fe=55.845)


def iso_to_species(isotopologue):
    """'1H2-16O' -> 'H2O', '48Ti-16O' -> 'TiO' (chemistry.py:13-21)."""
    species = ""
    for element in isotopologue.split('-'):
        for s in re.findall(r'\D+\d*', element):
            species += ''.join(s)
    return species if len(species) > 0 else isotopologue


def iso_to_mass(isotopologue):
    """Mass in atomic mass units: '1H2-16O' -> 18 (chemistry.py:24-37)."""
    mass = 0.0
    for element in isotopologue.split('-'):
        multiples = [x for x in re.split(r'\D', element) if len(x) > 0]
        if len(multiples) > 1:
            species_mass, multiplier = multiples
            mass += float(multiplier) * float(species_mass)
        elif len(multiples) == 1:
            mass += float(multiples[0])
    if mass != 0:
        return mass
    if isotopologue not in ATOM_MASS:
        raise KeyError(f"no atomic mass for {isotopologue!r}")
    return ATOM_MASS[isotopologue]


def chemistry(temperatures, pressures, species, return_vmr=False, m_bar=M_BAR_DEFAULT):
    """Mock-FastChem mass (and optionally volume) mixing ratios per species, shape of
    ``temperatures`` (chemistry.py:114-205 with Mock_FastChem, :207-246)."""
    T = np.atleast_1d(value(temperatures, "K"))
    m_bar = float(value(m_bar, "g"))
    mmr, vmr = {}, {}
    for iso in species:
        v = np.full(T.shape, MOCK_VMR)
        vmr[iso] = v
        mmr[iso] = v * (iso_to_mass(iso) * AMU / m_bar)
    if return_vmr:
        return mmr, vmr
    return mmr


class ChemistryTable:
    """Mass mixing ratios tabulated on (temperature, pressure) nodes, e.g. a FastChem run
    over a (T, p) grid: ``values`` is ``{species: array[n_T][n_p]}`` (or an array
    [n_species][n_T][n_p] in the opacity dict's species order), ``temperature`` in K and
    ``pressure`` in bar, both ascending.  The engine interpolates it at each layer's
    (T, p) every sweep — linear in T and in log10 p, clamped to the node range — the way the
    reference calls ``chemistry(T, p)`` inside every ``kappa`` (opacity.py:246-248)."""

    def __init__(self, values, temperature, pressure):
        self.temperature = np.asarray(value(temperature, "K"), dtype=np.float64)
        self.pressure = np.asarray(value(pressure, "bar"), dtype=np.float64)
        self.values = values
        if np.any(np.diff(self.temperature) <= 0) or np.any(np.diff(self.pressure) <= 0):
            raise ValueError("ChemistryTable nodes must be strictly ascending")

    def array(self, species):
        """[n_species][n_T][n_p] in the order of ``species``."""
        if isinstance(self.values, dict):
            v = np.array([np.asarray(self.values[n], dtype=np.float64) for n in species])
        else:
            v = np.asarray(self.values, dtype=np.float64)
        shape = (len(species), self.temperature.size, self.pressure.size)
        if v.shape != shape:
            raise ValueError(f"chemistry table must be {shape}, got {v.shape}")
        return np.ascontiguousarray(v)


# ------------------------------------------------------------------ chemistry providers
# The reference's kappa calls ``chemistry(T, p, opacities.keys(), m_bar=m_bar)`` for every layer
# of every sweep (opacity.py:246-248) — frei.chemistry.chemistry, which runs FastChem when
# pyfastchem imports and the mock otherwise (chemistry.py:142-153).  A provider is any callable
# on that signature returning {isotopologue: mass mixing ratio array}.  The engine takes one as
# ``chemistry=`` (Engine, Grid.load_opacities, the emit/absorb/kappa shims) and feeds the
# provider's own values to the opacity sum, never the built-in mock.

# temperatures at which a provider is probed for T dependence: 50 K .. 10,000 K
PROBE_T = np.geomspace(50.0, 1.0e4, 17)
# a provider whose mixing ratios move by less than this (relative) over PROBE_T is taken as
# T-independent: the reference's own mock returns 1.5e-3 n/n, equal to an ulp or two
PROBE_RTOL = 1e-12


def provider_mmr(provider, temperatures, pressures_bar, species, m_bar):
    """Mass mixing ratios [n_species][n] of ``provider`` at the points (T[i], p[i]), called as
    the reference calls its chemistry (opacity.py:246-248): temperatures in K and pressures in
    bar as astropy Quantities when astropy is importable (the reference's own environment),
    plain arrays otherwise; ``m_bar`` in g likewise."""
    T = np.atleast_1d(np.asarray(temperatures, dtype=np.float64))
    p = np.atleast_1d(np.asarray(pressures_bar, dtype=np.float64))
    try:
        import astropy.units as u
        args, mb = (T * u.K, p * u.bar), float(m_bar) * u.g
    except ImportError:
        args, mb = (T, p), float(m_bar)
    out = provider(*args, list(species), m_bar=mb)
    rows = []
    for iso in species:
        if iso not in out:
            raise KeyError(f"chemistry provider returned no mixing ratio for {iso!r} "
                           "(the reference's kappa would fail the same way)")
        v = out[iso]
        v = getattr(v, "value", v)            # a dimensionless Quantity
        rows.append(np.broadcast_to(np.asarray(v, dtype=np.float64), T.shape))
    return np.array(rows)


def fixed_provider_mmr(provider, species, pressures_bar, m_bar, temperatures=PROBE_T,
                       rtol=PROBE_RTOL):
    """[n_species][n_layers] when ``provider`` does not depend on temperature at the layer
    pressures (probed at ``temperatures``, relative spread <= ``rtol``), else None."""
    p = np.asarray(pressures_bar, dtype=np.float64)
    T = np.asarray(temperatures, dtype=np.float64)
    v = provider_mmr(provider, np.repeat(T, p.size), np.tile(p, T.size), species, m_bar)
    v = v.reshape(len(species), T.size, p.size)
    ref = v[:, T.size // 2, :]
    if np.all(np.abs(v - ref[:, None, :]) <= rtol * np.abs(ref[:, None, :])):
        return np.ascontiguousarray(ref)
    return None
