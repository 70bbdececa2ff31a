"""Batched atmospheres on one GPU (BASELINE config C5: grid sweeps).

The reference has no batch API: a grid sweep is a loop over independent ``Grid`` objects,
each running ``emission_spectrum`` (core.py:109-338).  :class:`BatchEngine` runs such a loop
as one device context (``frei_ctx_create_batch``): the atmospheres share the wavelength and
pressure grids and the opacity tables; each has its own temperatures, gravity and mixing
ratios.  Every sweep is one launch over (wavelength block, atmosphere); the per-atmosphere
species contraction is one dense product per layer on fp64 MFMA (K7).  Across GPUs the
atmospheres are sharded with no exchange.
"""
import ctypes

import numpy as np

from . import _native as N
from .chemistry import chemistry
from .constants import BAR, K_B, M_BAR_DEFAULT, UM
from .engine import EMIT, Engine, f_toa, planck_prefactor, trapz_weights
from .opacity import sigma_scattering
from .units import scalar, value

__all__ = ["BatchEngine", "batched_emission_spectra"]


class BatchEngine:
    """``n_atm`` atmospheres on ``device``: ``g`` [n_atm] (cm s^-2), ``mmr``
    [n_atm][n_species][n_layers], ``F_toa`` [n_lam] shared or [n_atm][n_lam] per atmosphere;
    wavelengths, pressures (bar, descending), opacities and m_bar are shared (as in a grid of
    Planets that differ in T, g, metallicity and irradiation)."""

    def __init__(self, lam_um, p_bar, opacities, g, mmr=None, m_bar=M_BAR_DEFAULT, F_toa=None,
                 device=0):
        lib = N.lib()
        self.lam_um = np.asarray(value(lam_um, "um"), dtype=float)
        self.p_bar = np.asarray(value(p_bar, "bar"), dtype=float)
        self.g = N.f64(np.atleast_1d(np.asarray(g, dtype=float)))
        self.n_atm = self.g.size
        self.m_bar = scalar(m_bar, "g")
        self.names = list(opacities)
        self.n_layers = self.p_bar.size
        self.n_lam = self.lam_um.size
        self.device = device
        lam_cm = self.lam_um * UM
        c1 = N.f64(planck_prefactor(lam_cm))
        lk = N.f64(lam_cm * K_B)
        sig = N.f64(sigma_scattering(self.lam_um, self.m_bar))
        ft = N.f64(f_toa(self.lam_um) if F_toa is None else value(F_toa, "erg / (s cm3)"))
        ft_atm = None
        if ft.ndim == 2:     # one F_TOA per atmosphere (planets around different stars)
            ft_atm = N.f64(np.broadcast_to(ft, (self.n_atm, self.n_lam)))
            ft = N.f64(ft_atm[0])
        wtr = N.f64(trapz_weights(lam_cm))
        p_cgs = N.f64(self.p_bar * BAR)
        ctx = ctypes.c_void_p()
        N.check(lib.frei_ctx_create_batch(ctypes.byref(ctx), device, self.n_layers, self.n_lam,
                                          len(self.names), self.n_atm))
        self._ctx = ctx
        N.check(lib.frei_set_grid(ctx, N.dptr(c1), N.dptr(lk), N.dptr(sig), N.dptr(ft),
                                  N.dptr(wtr), N.dptr(p_cgs), float(self.g[0]), self.m_bar))
        if self.n_atm > 1:
            N.check(lib.frei_set_gravity(ctx, N.dptr(self.g)))
            if ft_atm is not None:
                N.check(lib.frei_set_ftoa_batch(ctx, N.dptr(ft_atm)))
        self.lo = 0  # the whole wavelength grid
        # tables: the single-atmosphere engine's upload paths (shared by every atmosphere)
        for s, name in enumerate(self.names):
            Engine._set_table(self, s, opacities[name], slice(0, self.n_lam))
        if mmr is None:
            T0 = np.full(self.n_layers, 1000.0)
            mm = chemistry(T0, self.p_bar, self.names, m_bar=self.m_bar)
            mmr = np.array([mm[nm] for nm in self.names])
        self.mmr = N.f64(np.broadcast_to(np.asarray(mmr, dtype=float),
                                         (self.n_atm, len(self.names), self.n_layers)))
        N.check(lib.frei_set_mmr(ctx, N.dptr(self.mmr)))

    def close(self):
        if getattr(self, "_ctx", None):
            N.lib().frei_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, T_init, n_timesteps=1, n_zero_crossings=2, convergence_dT=3.0, alpha=1.0):
        """Every atmosphere's emission_spectrum (core.py:233-338) -> dict(spectra [n_atm]
        [n_lam], final_T [n_atm][n_layers], n_iter [n_atm])."""
        T = N.f64(np.broadcast_to(np.asarray(T_init, dtype=float), (self.n_atm, self.n_layers)))
        n_iter = (ctypes.c_int * self.n_atm)()
        T_final = np.empty((self.n_atm, self.n_layers))
        spectra = np.empty((self.n_atm, self.n_lam))
        N.check(N.lib().frei_run_batch(self._ctx, N.dptr(T), int(n_timesteps),
                                       int(n_zero_crossings), float(convergence_dT),
                                       float(alpha), n_iter, N.dptr(T_final),
                                       N.dptr(spectra)))
        return dict(spectra=spectra, final_T=T_final, n_iter=np.array(list(n_iter)))

    # fixed-work driver pieces (benchmarks)
    def state_init(self, T_init):
        T = N.f64(np.broadcast_to(np.asarray(T_init, dtype=float), (self.n_atm, self.n_layers)))
        N.check(N.lib().frei_state_init(self._ctx, N.dptr(T)))

    def iterate(self, n, n_zero_crossings=-1, convergence_dT=3.0, alpha=1.0):
        N.check(N.lib().frei_iterate(self._ctx, int(n), int(n_zero_crossings),
                                     float(convergence_dT), float(alpha)))

    def synchronize(self):
        N.check(N.lib().frei_synchronize(self._ctx))

    def timing(self, on):
        N.check(N.lib().frei_timing_enable(self._ctx, 1 if on else 0))

    def timing_read(self):
        ms, n = ctypes.c_double(0), ctypes.c_int(0)
        N.check(N.lib().frei_timing_read(self._ctx, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def setup_timing(self):
        return Engine.setup_timing(self)

    def set_option(self, name, value):
        return Engine.set_option(self, name, value)

    def contract_timing(self):
        return Engine.contract_timing(self)

    def get_fluxes(self):
        up = np.empty((self.n_atm, self.n_layers, self.n_lam))
        down = np.empty_like(up)
        N.check(N.lib().frei_get_fluxes(self._ctx, N.dptr(up), N.dptr(down)))
        return up, down

    path = Engine.path


def batched_emission_spectra(grids, n_timesteps=1, n_zero_crossings=2, convergence_dT=3.0,
                             device=0):
    """Grid.emission_spectrum for a list of Grids that share wavelengths, pressures and
    opacity tables (a grid sweep over T, g and metallicity), as one batched device run.
    Returns [(Spectrum, final_T, n_iter)] in the order of ``grids``."""
    from .core import F_TOA, Spectrum
    g0 = grids[0]
    for gr in grids[1:]:
        if not (np.array_equal(gr.lam, g0.lam) and np.array_equal(gr.pressures, g0.pressures)):
            raise ValueError("batched grids must share wavelengths and pressures")
        if gr.opacities is not g0.opacities:
            raise ValueError("batched grids must share one opacity dict")
        if gr.planet.alpha != g0.planet.alpha or gr.planet.m_bar != g0.planet.m_bar:
            raise ValueError("batched grids must share alpha and m_bar")
    names = list(g0.opacities)
    mmrs = []
    for gr in grids:
        if gr.mmr is not None:
            mmrs.append(np.broadcast_to(np.asarray(gr.mmr, dtype=float),
                                        (len(names), gr.pressures.size)))
        else:
            mm = chemistry(np.full(gr.pressures.size, 1000.0), gr.pressures, names,
                           m_bar=gr.planet.m_bar)
            mmrs.append(np.array([mm[n] for n in names]))
    pl = g0.planet
    # each planet's own irradiation (core.py:262): one F_TOA per atmosphere when they differ
    ft = np.array([F_TOA(g0.lam, T_star=gr.planet.T_star, a_rstar=gr.planet.a_rstar)
                   for gr in grids])
    if all(np.array_equal(f, ft[0]) for f in ft[1:]):
        ft = ft[0]
    eng = BatchEngine(g0.lam, g0.pressures, g0.opacities, [gr.planet.g for gr in grids],
                      mmr=np.array(mmrs), m_bar=pl.m_bar, F_toa=ft, device=device)
    try:
        out = eng.run(np.array([gr.init_temperatures for gr in grids]), n_timesteps,
                      n_zero_crossings, scalar(convergence_dT, "K"), pl.alpha)
    finally:
        eng.close()
    return [(Spectrum(out["spectra"][m], g0.lam), out["final_T"][m], int(out["n_iter"][m]))
            for m in range(len(grids))]
