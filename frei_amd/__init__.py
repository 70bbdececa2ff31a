"""frei_amd — MI355X-native (gfx950) two-stream radiative-transfer engine.

Drop-in for bmorris3/frei's hot path (per-wavelength two-stream flux recurrence,
species-summed opacity assembly, radiative-equilibrium T-P loop): the public names of
``frei`` below keep their signatures; the compute runs in hand-written HIP kernels
(``frei_amd/csrc``) behind the C ABI of ``include/frei_hip.h``.
"""
from .batch import BatchEngine, batched_emission_spectra
from .binning import BinnedTable, CrossSection, open_cross_section
from .chemistry import ChemistryTable, chemistry, iso_to_mass, iso_to_species
from .core import (B_star, F_TOA, Grid, Planet, Spectrum, contribution_function,
                   effective_temperature,
                   effective_temperature_milne, effective_temperature_planck, wavelength_grid)
from .engine import Engine, balanced_edges, partition, trapz_weights
from .opacity import (OpacityTable, SeparableTable, binned_opacity, kappa,
                      load_example_opacity, rayleigh_H2, rayleigh_He)
from .tp import pressure_grid, temperature_grid
from .twostream import BB, E, absorb, emit, propagate_fluxes

__version__ = "0.1.0"

__all__ = ["Planet", "Grid", "Spectrum", "effective_temperature", "wavelength_grid", "F_TOA",
           "B_star", "kappa", "load_example_opacity", "OpacityTable", "SeparableTable",
           "binned_opacity", "rayleigh_H2", "rayleigh_He", "chemistry", "iso_to_species",
           "iso_to_mass", "pressure_grid", "temperature_grid", "propagate_fluxes", "emit",
           "absorb", "BB", "E", "Engine", "balanced_edges", "partition", "trapz_weights", "CrossSection",
           "BinnedTable", "open_cross_section", "contribution_function", "BatchEngine",
           "batched_emission_spectra", "ChemistryTable"]
