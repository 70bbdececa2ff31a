"""User API: Planet, Grid, emission_spectrum, effective temperature (frei/core.py).

``Grid.emission_spectrum`` runs the whole radiative-equilibrium T-P loop on the GPU
(frei_run: device-resident sweeps, bolometric reductions, dT, convergence test).
"""
import numpy as np

from .constants import A_RSTAR_HOT_JUPITER, G_JUPITER, M_BAR_HOT_JUPITER, SIGMA_SB, UM
from .engine import Engine, f_toa
from .tp import pressure_grid, temperature_grid
from .twostream import BB
from .units import scalar, value

__all__ = ["Grid", "Planet", "Spectrum", "effective_temperature", "wavelength_grid", "F_TOA",
           "B_star", "contribution_function"]


def wavelength_grid(min_micron=0.5, max_micron=10, n_bins=500, lam=None):
    """Log-spaced wavelengths (µm), bin edges and resolution (core.py:34-45; Q14)."""
    if lam is None:
        lam = np.logspace(np.log10(min_micron), np.log10(max_micron), n_bins)
    lam = np.asarray(value(lam, "um"), dtype=float)
    d0 = lam[1] - lam[0]
    wl_bins = np.concatenate([[lam.min() - d0], lam]) + d0 / 2
    m = lam.shape[0] // 2
    R = float(lam[m] / (lam[m + 1] - lam[m]))
    return lam, wl_bins, R


def F_TOA(lam, T_star=5800.0, f=2 / 3, a_rstar=A_RSTAR_HOT_JUPITER):
    """Irradiation at the top of the atmosphere, erg s^-1 cm^-3 (core.py:48-55)."""
    return f_toa(value(lam, "um"), scalar(T_star, "K"), f, a_rstar)


def B_star(T_star, lam):
    """Stellar blackbody (core.py:58-62)."""
    return BB(T_star)(lam)


class Planet:
    """Planetary system (core.py:65-106). m_bar in g, g in cm s^-2, T_star in K."""

    def __init__(self, a_rstar, m_bar, g, T_star, alpha):
        self.a_rstar = float(a_rstar)
        self.m_bar = scalar(m_bar, "g")
        self.g = scalar(g, "cm / s2")
        self.T_star = scalar(T_star, "K")
        self.alpha = alpha

    @classmethod
    def from_hot_jupiter(cls):
        """M_J, R_J, m_bar = 2.4 m_p, g = g_J, T_star = 5800 K, a = 0.03 AU (core.py:92-106)."""
        return cls(a_rstar=A_RSTAR_HOT_JUPITER, m_bar=M_BAR_HOT_JUPITER, g=G_JUPITER,
                   T_star=5800.0, alpha=1)


class Spectrum:
    """Minimal Spectrum1D stand-in: ``flux`` (erg s^-1 cm^-3) on ``wavelength`` (µm)."""

    def __init__(self, flux, spectral_axis):
        self.flux = np.asarray(flux)
        self.spectral_axis = np.asarray(spectral_axis)

    @property
    def wavelength(self):
        return self.spectral_axis


class Grid:
    """Grid over temperatures, pressures and wavelengths (core.py:109-338).

    Units: wavelengths µm, pressures bar, temperatures K.  ``device`` selects the GPU."""

    def __init__(self, planet, lam=None, pressures=None, init_temperatures=None,
                 lam_min=0.5, lam_max=10, n_wl_bins=500, P_toa=1e-6, P_boa=200,
                 n_layers=30, T_ref=2300, P_ref=0.1, alpha=0.1, device=0):
        self.planet = planet
        if lam is None:
            self.lam, self.wl_bins, self.R = wavelength_grid(
                min_micron=scalar(lam_min, "um"), max_micron=scalar(lam_max, "um"),
                n_bins=n_wl_bins)
        else:
            self.lam, self.wl_bins, self.R = wavelength_grid(lam=lam)
        if pressures is None:
            self.pressures = pressure_grid(n_layers=n_layers,
                                           P_toa=np.log10(scalar(P_toa, "bar")),
                                           P_boa=np.log10(scalar(P_boa, "bar")))
        else:
            self.pressures = np.asarray(value(pressures, "bar"), dtype=float)
        if init_temperatures is None:
            self.init_temperatures = temperature_grid(self.pressures, T_ref, P_ref, alpha)
        else:
            self.init_temperatures = np.asarray(value(init_temperatures, "K"), dtype=float)
        self.opacities = None
        self.mmr = None
        self.chemistry = None
        self.device = device
        self._engine = None
        self._last_dtaus = None

    def __repr__(self):
        return (f"<Grid in T=[{self.init_temperatures[0]:.0f}...{self.init_temperatures[-1]:.0f}] K, "
                f"p=[{self.pressures[0]:.2g}...{self.pressures[-1]:.2g}] bar, "
                f"lam=[{self.lam[0]}...{self.lam[-1]}] um>")

    def load_opacities(self, species=None, path=None, opacities=None, client=None,
                       force_reload=False, groupies=False, mmr=None, cross_sections=None,
                       chemistry=None):
        """Attach opacity tables (core.py:198-231).  ``opacities`` is the reference's dict
        of (pressure, temperature, wavelength) tables; otherwise high-resolution
        cross-sections (files at ``path`` or ``cross_sections``) are binned on the GPU
        straight into the engine's tables (opacity.py:66-170).  The mixing ratios come from
        ``chemistry`` — a provider on the reference's ``chemistry(T, p, species, m_bar=...)``
        signature, called wherever the reference's kappa calls it (opacity.py:246-248; the
        drop-in passes frei's own) — or ``mmr`` (per-species, per-layer
        arrays or a ChemistryTable); with neither, the reference's mock."""
        if (self.opacities is None and opacities is None) or force_reload:
            from .binning import binned_opacity
            self.opacities = binned_opacity(self.init_temperatures, self.pressures,
                                            self.wl_bins, self.lam, species=species,
                                            path=path, groupies=groupies,
                                            cross_sections=cross_sections, device=self.device)
        else:
            self.opacities = opacities
        if mmr is not None and chemistry is not None:
            raise ValueError("pass either mmr or a chemistry provider, not both")
        self.mmr = mmr
        self.chemistry = chemistry
        self._close_engine()
        return self.opacities

    def _close_engine(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None
        self._last_dtaus = None   # its device copy went with the engine

    def engine(self):
        if self._engine is None:
            pl = self.planet
            self._engine = Engine(self.lam, self.pressures, self.opacities, g=pl.g,
                                  m_bar=pl.m_bar,
                                  F_toa=F_TOA(self.lam, T_star=pl.T_star, a_rstar=pl.a_rstar),
                                  mmr=self.mmr, chemistry=self.chemistry, device=self.device)
        return self._engine

    def emission_spectrum(self, n_timesteps=1, n_zero_crossings=2, convergence_dT=3.0):
        """Emission spectrum after iterating toward radiative equilibrium (core.py:233-338)
        -> (spectrum, final_temps, temperature_history, dtaus)."""
        if self.opacities is None:
            raise ValueError("Must load opacities before computing emission spectrum.")
        if n_timesteps < 1:
            raise ValueError("n_timesteps must be >= 1")
        out = self.engine().run(self.init_temperatures, n_timesteps=n_timesteps,
                                n_zero_crossings=n_zero_crossings,
                                convergence_dT=scalar(convergence_dT, "K"),
                                alpha=self.planet.alpha)
        th = out["temp_hist"]
        th = th.T[th[0] != 0].T   # core.py:320-321
        self._last_dtaus = out["dtaus"]
        return (Spectrum(out["spectrum"], self.lam), out["final_T"], th, out["dtaus"])

    def contribution_function(self, final_temps, dtaus=None):
        """Contribution function of the last emission_spectrum (plot.py:63-79)."""
        return contribution_function(self, self._last_dtaus if dtaus is None else dtaus,
                                     final_temps)

    def emission_dashboard(self, *args, **kwargs):
        raise NotImplementedError("plotting is out of scope for the MI355X engine (SURVEY.md §2)")


def _post_engine(grid, dtaus):
    """The grid's engine and the dtaus argument for the device: None when ``dtaus`` is the
    array the last emission_spectrum returned (its device copy is used)."""
    eng = grid.engine()
    same = dtaus is getattr(grid, "_last_dtaus", None)
    return eng, (None if same else np.asarray(dtaus, dtype=float))


def effective_temperature_milne(grid, spec, dtaus, final_temps):
    """Photosphere temperature from Milne's tau ~ 2/3 (core.py:386-405).  The per-wavelength
    np.interp over layers runs on the GPU (frei_milne_pressure); the weighted mean and the
    final interpolation are O(n_lambda) host work, as in the reference."""
    lam = np.asarray(grid.lam)
    p = np.asarray(grid.pressures)
    eng, d = _post_engine(grid, dtaus)
    pressure_milne = eng.milne_pressure(p, d)
    # weights: F_lambda -> lambda F_lambda (erg s^-1 cm^-2, astropy spectral_density)
    lam_flux = np.asarray(spec.flux) * (lam * UM)
    return np.interp(np.average(pressure_milne, weights=lam_flux), p[::-1],
                     np.asarray(final_temps)[::-1])


def contribution_function(grid, dtaus, final_temps):
    """Normalised contribution function of the final atmosphere (plot.py:63-79), computed
    on the GPU: array (n_layers, n_lambda), rows bottom-first like ``grid.pressures`` (the
    reference plots ``cf[::-1]``)."""
    eng, d = _post_engine(grid, dtaus)
    return eng.contribution(np.asarray(grid.pressures), np.asarray(final_temps), d)


def effective_temperature_planck(grid, spec):
    """Stefan-Boltzmann inversion of the bolometric flux (core.py:408-414)."""
    lam_cm = np.asarray(grid.lam) * UM
    f = np.asarray(spec.flux)
    bol = np.sum(np.diff(lam_cm) * (f[1:] + f[:-1]) / 2.0)
    return (bol / SIGMA_SB) ** 0.25


def effective_temperature(grid, spec, dtaus, final_temps):
    """Mean of the Milne and Stefan-Boltzmann estimates, K (core.py:417-439)."""
    return float(np.mean([effective_temperature_milne(grid, spec, dtaus, final_temps),
                          effective_temperature_planck(grid, spec)]))
