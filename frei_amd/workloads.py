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


def c3_chemistry(w, n_T=14, n_p=9):
    """A T-dependent chemistry table for the C3 species (frei_amd.ChemistryTable): mass
    mixing ratios on (T, p) nodes around each species' median C3 value, half of the species
    falling with T and half rising (a tanh around 1500 K, weak log-p slope).  Synthetic: the
    reference's FastChem is third-party and absent."""
    from .chemistry import ChemistryTable
    cT = np.linspace(300.0, 4000.0, n_T)
    cp = np.logspace(-7, 3, n_p)
    x = np.tanh((cT[:, None] - 1500.0) / 400.0) + 0.05 * np.log10(cp)[None, :]
    vals = {n: float(np.median(w["mmr"][s])) * 10 ** (0.5 * (-1) ** s * x)
            for s, n in enumerate(w["names"])}
    return ChemistryTable(vals, cT, cp)


def c3_provider(w):
    """A T-dependent chemistry *provider* for the C3 species on the reference's chemistry
    signature, ``chemistry(temperatures, pressures, species, return_vmr=False, m_bar=...)``
    (frei/chemistry.py:114-116; pressures in bar): c3_chemistry's law evaluated at the query
    points.  It stands in for FastChem on the path the drop-in takes (``chemistry=``, evaluated
    on the host between sweeps); FastChem itself is third-party and absent."""
    med = {n: float(np.median(w["mmr"][s])) for s, n in enumerate(w["names"])}
    sign = {n: (-1) ** s for s, n in enumerate(w["names"])}

    def chemistry(temperatures, pressures, species, return_vmr=False, m_bar=None):
        T = np.atleast_1d(np.asarray(getattr(temperatures, "value", temperatures), dtype=float))
        p = np.atleast_1d(np.asarray(getattr(pressures, "value", pressures), dtype=float))
        x = np.tanh((T - 1500.0) / 400.0) + 0.05 * np.log10(p)
        mmr = {n: med[n] * 10 ** (0.5 * sign[n] * x) for n in species}
        return (mmr, dict(mmr)) if return_vmr else mmr
    return chemistry


def bytes_per_update(n_species, write_dtau=False, live_only=False):
    """Algorithmic HBM bytes per (layer, wavelength) flux update:
    stale opposite-stream read 8 + two flux writes 16 + two T-bracket rows per species.
    Inside the T-P loop (live_only) one of the two flux rows per step is a dead store that
    the engine skips, so 8 + 8 + 16 S."""
    return 8 + (8 if live_only else 16) + 16 * n_species + (8 if write_dtau else 0)


def binning_workload(n_layers=60, n_lam=500_000, T_ref=1500.0, spacing_cm=0.01,
                     n_T_src=20, n_p_src=12):
    """K6 benchmark: one species' DACE-like cross-section (float32, wavenumber spacing
    ``spacing_cm`` cm^-1 over 1000-20000 cm^-1, i.e. 0.5-10 µm; ``n_T_src`` x ``n_p_src``
    nodes 500-4300 K x 1e-6-100 bar) binned onto the C3 grid with the reference's output
    shape: every (grid T, grid p) node (n_layers x n_layers rows of n_lam bins)."""
    lam, wl_bins, _ = wavelength_grid(0.5, 10, n_lam)
    p = pressure_grid(n_layers, -6, np.log10(200))
    T0 = temperature_grid(p, T_ref, 0.1, 0.1)
    wlen = np.arange(1000, 20000, spacing_cm)
    wl_hi = (1 / wlen / 1e-4)[1:][::-1]                 # opacity.py:409-414
    T_src = np.linspace(500.0, 4300.0, n_T_src)
    p_src = np.logspace(-6, 2, n_p_src)
    return dict(lam=lam, wl_bins=wl_bins, p=p, T0=T0, wl_hi=wl_hi, T_src=T_src, p_src=p_src)


def nearest_index(nodes, targets):
    """Nearest-node selection of the binning plan (interp 'nearest', ties to the lower node,
    extrapolating): for accounting the rows a binning launch reads."""
    nodes = np.asarray(nodes, dtype=float)
    order = np.argsort(nodes, kind="stable")
    x = nodes[order]
    if x.size == 1:
        return np.full(np.size(targets), order[0])
    h = x / 2.0
    return order[np.clip(np.searchsorted(h[1:] + h[:-1], targets, side="left"), 0, x.size - 1)]


def binning_bytes(w, groupies=True):
    """Algorithmic HBM bytes of one binning launch: every selected source row read once over
    the binned wavelength range (float32), every destination table row written once
    (float64), the per-bin plan (start, end, width: 24 B per bin) read once; the exact
    mode also reads the float64 dx stream once."""
    wl, b = w["wl_hi"], w["wl_bins"]
    lo = np.searchsorted(wl, b[0], side="right")
    hi = np.searchsorted(wl, b[-1], side="left")
    P = int(hi - lo)
    U = len({(t, q) for t in nearest_index(w["T_src"], w["T0"])
             for q in nearest_index(w["p_src"], w["p"])})
    D = w["T0"].size * w["p"].size
    n = w["lam"].size
    reads = U * P * 4 + 24 * n + (0 if groupies else 8 * P)
    writes = D * n * 8
    return dict(bytes=reads + writes, source_rows=U, points=P, dest_rows=D, n_bins=n)
