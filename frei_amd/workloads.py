"""Synthetic benchmark workloads of SURVEY.md §8(d) (no network: no DACE tables).

C3: hot Jupiter, 60 layers x 500k wavelengths (0.5-10 µm), species H2O/CO/CO2/CH4/Na/K
plus two collision-induced (CIA) tables H2-H2 and H2-He whose per-layer weights are
supplied (the reference has no CIA; parity for them is pinned to the same table path).
Tables are separable log-normal line forests (continuum + 2000 lines of ~2-bin width,
strengths log-normal), scaled by (T/1000 K)^0.5 (p/1 bar)^0.1 and clipped to
[1e-4, 1e3] cm^2 g^-1, on n_T temperature nodes spanning 0.8 min(T0)..1.2 max(T0).
"""
import numpy as np

from .chemistry import chemistry
from .constants import M_BAR_HOT_JUPITER
from .core import wavelength_grid
from .tp import pressure_grid, temperature_grid

C3_SPECIES = ["1H2-16O", "12C-16O", "12C-16O2", "12C-1H4", "Na", "K", "H2-H2", "H2-He"]


def line_forest(lam_um, seed, n_lines=2000, width_bins=2.0):
    """log10-space continuum + Gaussian lines, returned as linear opacity (cm^2 g^-1)."""
    rng = np.random.default_rng(seed)
    n = lam_um.size
    x = np.log(lam_um)
    logk = -1.0 + 0.8 * np.sin(2.1 * x + seed) + 0.3 * np.cos(5.3 * x)
    centres = rng.integers(0, n, n_lines)
    strengths = rng.lognormal(0.0, 1.0, n_lines)
    half = int(6 * width_bins)
    offs = np.arange(-half, half + 1)
    prof = np.exp(-0.5 * (offs / width_bins) ** 2)
    for c0, s0 in zip(centres, strengths):
        idx = c0 + offs
        ok = (idx >= 0) & (idx < n)
        logk[idx[ok]] += s0 * prof[ok]
    return 10 ** logk


def c3(n_layers=60, n_lam=500_000, n_T=16, T_ref=1500.0, species=None, seed=42):
    """Return dict(lam, p, T0, T_nodes, names, base[S][n_lam], fp[S][n_p], fT[S][n_T], mmr)."""
    names = list(C3_SPECIES if species is None else species)
    lam, _, _ = wavelength_grid(0.5, 10, n_lam)
    p = pressure_grid(n_layers, -6, np.log10(200))
    T0 = temperature_grid(p, T_ref, 0.1, 0.1)
    T_nodes = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), n_T)
    base = np.array([line_forest(lam, seed + s) for s in range(len(names))])
    fp = np.array([(p / 1.0) ** 0.1 for _ in names])
    fT = np.array([(T_nodes / 1000.0) ** 0.5 for _ in names])
    mol = [n for n in names if n not in ("H2-H2", "H2-He")]
    mm = chemistry(T0, p, mol, m_bar=M_BAR_HOT_JUPITER)
    rows = []
    for n in names:
        if n == "H2-H2":
            rows.append(1e-3 * np.minimum(1.0, p / 1.0))
        elif n == "H2-He":
            rows.append(2e-4 * np.minimum(1.0, p / 1.0))
        else:
            rows.append(mm[n])
    return dict(lam=lam, p=p, T0=T0, T_nodes=T_nodes, names=names, base=base, fp=fp, fT=fT,
                mmr=np.array(rows))


def bytes_per_update(n_species, write_dtau=False, live_only=False):
    """Algorithmic HBM bytes per (layer, wavelength) flux update:
    stale opposite-stream read 8 + two flux writes 16 + two T-bracket rows per species.
    Inside the T-P loop (live_only) one of the two flux rows per step is a dead store that
    the engine skips, so 8 + 8 + 16 S."""
    return 8 + (8 if live_only else 16) + 16 * n_species + (8 if write_dtau else 0)
