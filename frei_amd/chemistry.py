"""Mass mixing ratios (frei/chemistry.py:114-246).

FastChem (``pyfastchem``, third-party C++, unpinned) is not part of this engine; like the
reference when pyfastchem is absent (chemistry.py:142-153) the built-in mock is used:
every species has VMR = 1.5e-3 (chemistry.py:243), mmr = VMR * mass / m_bar.  The
engine takes per-layer mmr arrays, so a real chemistry provider can be plugged in by
passing ``mmr=`` to :class:`frei_amd.engine.Engine` / ``Grid.load_opacities``; a provider
whose abundances depend on temperature (FastChem's equilibrium chemistry) is passed as a
:class:`ChemistryTable` — its output tabulated on (T, p) nodes — and the device re-evaluates
every layer's mmr at the layer's current temperature each sweep (frei_set_chemistry).
"""
import re

import numpy as np

from .constants import AMU, M_BAR_DEFAULT
from .units import value

__all__ = ["chemistry", "iso_to_species", "iso_to_mass", "ChemistryTable"]

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
