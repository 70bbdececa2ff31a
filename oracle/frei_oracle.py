"""CPU oracle — TEST INFRASTRUCTURE ONLY, never part of the product path.

A unit-free (cgs) NumPy restatement of bmorris3/frei's hot path, used as the
parity checker for the HIP engine.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it; ``frei_amd`` never does.

Pinning: every function here is checked against golden vectors produced by
running the reference itself in the build container (``tests/golden/make_goldens.py``,
reference imported through the SURVEY.md Appendix B stand-ins), see
``tests/test_oracle_golden.py``.  It follows the reference operation order,
including its quirks.

Units: wavelength cm (API takes µm like the reference), pressure dyn cm^-2
(API takes bar), temperature K, flux erg s^-1 cm^-3, opacity cm^2 g^-1.
"""
import numpy as np

# CODATA 2018 values as used by astropy 4.3.1 (the reference's units backend), cgs.
H = 6.62607015e-27             # erg s
C = 29979245800.0              # cm s^-1
K_B = 1.380649e-16             # erg K^-1
M_P = 1.67262192369e-24        # g
AMU = 1.6605390666e-24         # g
SIGMA_SB = 5.6703744191844314e-05  # erg cm^-2 s^-1 K^-4
BAR = 1e6                      # dyn cm^-2
M_BAR_DEFAULT = 2.4 * M_P      # twostream.py:23 / 208 default m_bar

N_REF_H2 = 2.68678e19          # opacity.py:23
N_REF_HE = 2.546899e19         # opacity.py:24

# periodictable masses for bare-atom species (chemistry.py:37)
ATOM_MASS = dict(H=1.00794, He=4.002602, C=12.0107, N=14.0067, O=15.9994, F=18.9984032,
                 Na=22.98977, Al=26.981538, Cl=35.453, K=39.0983, Ti=47.867, V=50.9415,
                 Cr=51.9961, Fe=55.845)


# ----------------------------------------------------------------- grids (core.py, tp.py)
def wavelength_grid(min_micron=0.5, max_micron=10, n_bins=500, lam=None):
    """core.py:34-45 (µm). Bin edges offset by the first linear spacing (Q14)."""
    if lam is None:
        lam = np.logspace(np.log10(min_micron), np.log10(max_micron), n_bins)
    lam = np.asarray(lam, dtype=float)
    d0 = lam[1] - lam[0]
    wl_bins = np.concatenate([[lam.min() - d0], lam]) + d0 / 2
    m = lam.shape[0] // 2
    R = float(lam[m] / (lam[m + 1] - lam[m]))
    return lam, wl_bins, R


def pressure_grid(n_layers=30, P_toa=-6, P_boa=1.1):
    """tp.py:10-33, bar, index 0 = bottom of atmosphere."""
    return np.logspace(P_toa, P_boa, n_layers)[::-1]


def temperature_grid(pressures, T_ref=2300.0, P_ref=0.1, alpha=0.1):
    """tp.py:36-62."""
    return T_ref * (np.asarray(pressures) / P_ref) ** alpha


# ----------------------------------------------------------------- physics kernels
def BB(T, lam_cm):
    """twostream.py:46-67: 2hc^2/lam^5 / expm1(hc/(lam k T))."""
    return 2 * H * C ** 2 / np.power(lam_cm, 5) / np.expm1(H * C / (lam_cm * K_B * T))


def F_TOA(lam_um, T_star=5800.0, f=2 / 3, a_rstar=6.450964670116429):
    """core.py:48-55."""
    lam_cm = np.asarray(lam_um) * 1e-4
    return f * a_rstar ** -2 * 1 / (2 * np.pi) * (np.pi * BB(T_star, lam_cm))


def E(omega_0, g_0=0.0):
    """twostream.py:70-94 (Deitrick 2020 Eqn 19)."""
    return np.where(omega_0 > 0.1,
                    1.225 - 0.1582 * g_0 - 0.1777 * omega_0 - 0.07465 * g_0 ** 2
                    + 0.2351 * omega_0 * g_0 - 0.05582 * omega_0 ** 2, 1)


def propagate_fluxes(lam_cm, F_1_up, F_2_down, T_1, T_2, delta_tau, omega_0=0.0, g_0=0.0):
    """twostream.py:97-177, same expression order (E re-evaluated as in the reference)."""
    omega_0 = np.asarray(omega_0, dtype=float).flatten()
    delta_tau = np.asarray(delta_tau, dtype=float).flatten()
    Ev = E(omega_0, g_0)
    T = np.exp(-2 * (Ev * (Ev - omega_0) * (1 - omega_0 * g_0)) ** 0.5 * delta_tau)
    r = ((Ev - omega_0) / Ev / (1 - omega_0 * g_0)) ** 0.5
    zeta_plus = 0.5 * (1 + r)
    zeta_minus = 0.5 * (1 - r)
    chi = zeta_minus ** 2 * T ** 2 - zeta_plus ** 2
    xi = zeta_plus * zeta_minus * (1 - T ** 2)
    psi = (zeta_minus ** 2 - zeta_plus ** 2) * T
    pi = np.pi * (1 - omega_0) / (Ev - omega_0)
    B1 = BB(T_1, lam_cm)
    B2 = BB(T_2, lam_cm)
    Bprime = (B1 - B2) / delta_tau
    den = 2 * Ev * (1 - omega_0 * g_0)
    F_2_up = 1 / chi * (psi * F_1_up - xi * F_2_down +
                        pi * (B2 * (chi + xi) - psi * B1 + Bprime / den * (chi - psi - xi)))
    F_1_down = 1 / chi * (psi * F_2_down - xi * F_1_up +
                          pi * (B1 * (chi + xi) - psi * B2 + Bprime / den * (xi + psi - chi)))
    return F_2_up, F_1_down


def propagate_error_bound(lam_cm, F_1_up, F_2_down, T_1, T_2, delta_tau, omega_0,
                          err_F1u=0.0, err_F2d=0.0, delta=np.finfo(float).eps, g_0=0.0):
    """First-order forward rounding-error bound of propagate_fluxes (test infrastructure).

    The reference formula is ill-conditioned for thin layers: ``1 - T**2`` and
    ``(B1 - B2)/dtau * (chi - psi - xi)`` cancel, so a relative perturbation
    ``delta`` of its operands (one ulp in ``exp``/``expm1``, or a relative error
    ``delta`` in T) moves F_2_up / F_1_down by up to ``delta * cond``.  ``err_*``
    are absolute error bounds already carried by the incoming fluxes; they are
    propagated through the recurrence coefficients psi/chi and xi/chi.
    Returns absolute bounds (e_F2u, e_F1d); tests allow |gpu - ref| <= K * bound.
    """
    w = np.asarray(omega_0, dtype=float)
    dtau = np.asarray(delta_tau, dtype=float)
    Ev = E(w, g_0)
    wg = 1 - w * g_0
    arg = 2 * (Ev * (Ev - w) * wg) ** 0.5 * dtau
    Tr = np.exp(-arg)
    r = ((Ev - w) / Ev / wg) ** 0.5
    zp, zm = 0.5 * (1 + r), 0.5 * (1 - r)
    chi = zm ** 2 * Tr ** 2 - zp ** 2
    xi = zp * zm * (1 - Tr ** 2)
    psi = (zm ** 2 - zp ** 2) * Tr
    pi = np.pi * (1 - w) / (Ev - w)
    B1, B2 = BB(T_1, lam_cm), BB(T_2, lam_cm)
    x1 = H * C / (lam_cm * K_B * T_1)
    x2 = H * C / (lam_cm * K_B * T_2)
    m1, m2 = np.abs(B1) * (1 + x1), np.abs(B2) * (1 + x2)
    den = 2 * Ev * wg
    mxi = np.abs(xi) + np.abs(zp * zm) * 2 * (1 + arg)
    cb = (np.abs((B1 - B2) / dtau / den) * (np.abs(chi) + np.abs(psi) + np.abs(xi))
          + (m1 + m2) / (dtau * den) * np.abs(chi - psi - xi))
    ic = np.abs(1 / chi)
    cu = ic * (np.abs(psi * F_1_up) + mxi * np.abs(F_2_down)
               + np.abs(pi) * (m2 * np.abs(chi + xi) + np.abs(psi) * m1 + cb))
    cd = ic * (np.abs(psi * F_2_down) + mxi * np.abs(F_1_up)
               + np.abs(pi) * (m1 * np.abs(chi + xi) + np.abs(psi) * m2 + cb))
    if np.any(np.asarray(g_0) != 0):
        # with g_0 != 0, E - omega_0 can cancel (it reaches 0 where the reference gives NaN):
        # a relative operand error delta becomes delta (|E| + |omega_0|) / |E - omega_0| in
        # E - omega_0, which feeds the transmission, zeta and pi
        with np.errstate(divide="ignore", invalid="ignore"):
            kE = (np.abs(Ev) + np.abs(w)) / np.abs(Ev - w)
        cu, cd = cu * np.maximum(kE, 1.0), cd * np.maximum(kE, 1.0)
    e_up = delta * cu + ic * (np.abs(psi) * err_F1u + np.abs(xi) * err_F2d)
    e_dn = delta * cd + ic * (np.abs(psi) * err_F2d + np.abs(xi) * err_F1u)
    return e_up, e_dn


def n_lambda_H2(lam_um):
    """opacity.py:173-177 (7.52e-11 cm^2 * lam^-2, lam in µm -> x1e8)."""
    return 13.58e-5 * (1 + (7.52e-11 * np.asarray(lam_um) ** -2) * 1e8) + 1


def n_lambda_He(lam_um):
    """opacity.py:180-184."""
    return 1e-8 * (2283 + (1.8102e13 / (1.5342e10 - np.asarray(lam_um) ** -2))) + 1


def _rayleigh(n, n_ref, lam_cm, m_bar):
    return (24 * np.pi ** 3 / n_ref ** 2 / lam_cm ** 4 * ((n ** 2 - 1) / (n ** 2 + 2)) ** 2 * 1) / m_bar


def rayleigh(lam_um, m_bar=M_BAR_DEFAULT):
    """rayleigh_H2 + rayleigh_He, opacity.py:187-200 and :233, cm^2 g^-1."""
    lam_um = np.asarray(lam_um, dtype=float)
    lam_cm = lam_um * 1e-4
    return (_rayleigh(n_lambda_H2(lam_um), N_REF_H2, lam_cm, m_bar)
            + _rayleigh(n_lambda_He(lam_um), N_REF_HE, lam_cm, m_bar))


# ----------------------------------------------------------------- chemistry (mock)
def iso_mass(iso):
    """chemistry.py:24-37 (atomic mass units)."""
    import re
    mass = 0.0
    for element in iso.split('-'):
        mult = [x for x in re.split(r'\D', element) if len(x) > 0]
        if len(mult) > 1:
            mass += float(mult[1]) * float(mult[0])
        elif len(mult) == 1:
            mass += float(mult[0])
    return mass if mass != 0 else ATOM_MASS[iso]


def mock_mmr(species, m_bar, vmr=1.5e-3):
    """chemistry.py:114-246 with the reference's own FastChem mock (VMR 1.5e-3, Q15)."""
    return np.array([vmr * (iso_mass(s) * AMU / m_bar) for s in species])


# ----------------------------------------------------------------- opacity tables / kappa
class Table:
    """(pressure [bar], temperature [K], wavelength) grid, like the reference's DataArray."""

    def __init__(self, values, pressure, temperature, wavelength=None):
        self.values = values if hasattr(values, "shape") and not isinstance(values, list) \
            and not isinstance(values, np.ndarray) else np.asarray(values, dtype=float)
        self.pressure = np.asarray(pressure, dtype=float)
        self.temperature = np.asarray(temperature, dtype=float)
        self.wavelength = wavelength


def _bracket(grid, x):
    """scipy RegularGridInterpolator._find_indices on an ascending grid (left searchsorted)."""
    i = int(np.searchsorted(grid, x)) - 1
    i = min(max(i, 0), grid.size - 2)
    y = (x - grid[i]) / (grid[i + 1] - grid[i])
    oob = (x < grid[0]) or (x > grid[-1])
    return i, y, oob


def _localized(coords, x):
    """xarray missing._localize: sort ascending, keep nearest-index +-2 nodes."""
    order = np.argsort(coords, kind="stable")
    c = coords[order]
    k = int(np.argmin(np.abs(c - x)))
    sl = np.arange(c.size)[slice(max(k - 2, 0), k + 2)]
    return c[sl], order[sl]


def _table_row(values, pi, ti):
    """values[pi, ti, :] — for a lazy SeparableValues only that row is formed (same arithmetic,
    elementwise, as the whole table)."""
    if isinstance(values, SeparableValues):
        return values.row(pi, ti)
    return values[pi, ti]


def interp_table(tab, T, p_bar):
    """xarray DataArray.interp(pressure, [temperature], linear, fill 0) at one point
    (opacity.py:250-263): interpn for 2-D, interp1d for the single-T case."""
    pc, pidx = _localized(tab.pressure, p_bar)
    if len(np.unique(tab.temperature)) > 1:
        tc, tidx = _localized(tab.temperature, T)
        ip, yp, oobp = _bracket(pc, p_bar)
        it, yt, oobt = _bracket(tc, T)
        if oobp or oobt:
            return np.zeros(tab.values.shape[-1])
        out = 0.
        for a, wa in ((ip, 1 - yp), (ip + 1, yp)):
            for b, wb in ((it, 1 - yt), (it + 1, yt)):
                out = out + _table_row(tab.values, pidx[a], tidx[b]) * (1. * wa * wb)
        return out
    vals = tab.values[pidx]
    # single unique temperature: scipy interp1d linear over pressure
    if p_bar < pc[0] or p_bar > pc[-1]:
        return np.zeros(vals.shape[-1])
    j = int(np.clip(np.searchsorted(pc, p_bar), 1, pc.size - 1))
    lo, hi = j - 1, j
    slope = (vals[hi, 0] - vals[lo, 0]) / (pc[hi] - pc[lo])
    return slope * (p_bar - pc[lo]) + vals[lo, 0]


def kappa(tables, T, p_bar, lam_um, m_bar, mmr=None):
    """opacity.py:203-269 -> (k, sigma), cm^2 g^-1.  k includes sigma (Q1).

    ``mmr``: per-species mass mixing ratios; default = the reference's mock chemistry."""
    sigma = rayleigh(lam_um, m_bar)
    names = list(tables)
    if mmr is None:
        mmr = mock_mmr(names, m_bar)
    ops = [mmr[s] * interp_table(tables[n], T, p_bar) for s, n in enumerate(names)]
    if len(ops) == 1:
        tot = ops[0]
    else:
        st = np.stack(ops, axis=0)
        tot = np.sum(np.where(np.isnan(st), 0.0, st), axis=0)  # xarray nansum (Q8)
    return tot + sigma, sigma


# ----------------------------------------------------------------- per-layer scalar physics
def trapz(y, x):
    """np.trapz (bolometric_flux, twostream.py:16-20)."""
    d = np.diff(x)
    return (d * (y[1:] + y[:-1]) / 2.0).sum()


def delta_z(T, p1, p2, g, m_bar):
    return (K_B * T) / (m_bar * g) * np.log(p1 / p2)


def c_p(m_bar, n_dof=5):
    return (2 + n_dof) / (2 * m_bar) * K_B


def rho_p(p1, p2, T1, g, m_bar):
    return ((p1 - p2) / g) / delta_z(T1, p1, p2, g, m_bar)


def delta_gamma(T1, T2, p1, p2, g, m_bar, n_dof=5):
    return (T1 - T2) / delta_z(T1, p1, p2, g, m_bar) - g / c_p(m_bar, n_dof)


def convective_flux(T1, T2, p1, p2, g, m_bar, n_dof=5, alpha=1):
    """twostream.py:273-287."""
    rho = rho_p(p1, p2, T1, g, m_bar)
    cp = c_p(m_bar, n_dof)
    lmix = alpha * K_B * T1 / (m_bar * g)
    dg = delta_gamma(T1, T2, p1, p2, g, m_bar, n_dof)
    if dg > 0:
        return rho * cp * lmix ** 2 * (g / T1) ** 0.5 * dg ** 1.5
    return 0.0


def layer_dT(Fb, T1, T2, p1, p2, g, m_bar, alpha):
    """div_bol_net_flux + delta_t_i + delta_temperature (twostream.py:23-43, 190-217).

    Fb = (F_2_up, F_2_down, F_1_up, F_1_down) bolometric (erg cm^-2 s^-1)."""
    F2u, F2d, F1u, F1d = Fb
    dF_rad = (F2u - F2d) - (F1u - F1d)
    dF_conv = convective_flux(T1, T2, p1, p2, g, m_bar, alpha=alpha)
    dz = delta_z(T1, p1, p2, g, m_bar)
    div = (dF_rad + dF_conv) / dz
    # delta_t_i (Malik 2017 Eqn 27-28)
    x = div * dz
    f = 1e5 / abs(x) ** 0.9 if x != 0 else 1
    dt_rad = c_p(m_bar) * p1 / SIGMA_SB / g / T1 ** 3
    dg = delta_gamma(T1, T2, p1, p2, g, m_bar)
    if dg > 0:
        dt = f * min(dt_rad, (T1 / g / dg) ** 0.5)
    else:
        dt = f * dt_rad
    # delta_temperature uses the default m_bar (Q7)
    m0 = M_BAR_DEFAULT
    return 1 / rho_p(p1, p2, T1, g, m0) / c_p(m0) * div * dt


# ----------------------------------------------------------------- sweeps
def _sweep(direction, tables, T, p_bar, lam_um, F_toa, g, m_bar, alpha, F_up, F_down, mmr_fn,
           err=None, bol_fn=None):
    """One emit/absorb sweep.  ``err``: optional dict {'up','down','delta'} of absolute
    error-bound rows tracked alongside the fluxes (propagate_error_bound)."""
    nL, nlam = F_up.shape
    lam_cm = lam_um * 1e-4
    p = p_bar * BAR
    dtaus = [np.ones(nlam)]
    dT = np.zeros(nL)
    layers = range(1, nL) if direction == "emit" else range(nL - 2, -1, -1)
    for i in layers:
        if direction == "emit" and i == nL - 1:
            p2b, T2 = p_bar[i] * p_bar[-2] / p_bar[-3], T[i]
        else:
            p2b, T2 = p_bar[i + 1], T[i + 1]
        p1b, T1 = p_bar[i], T[i]
        k, sigma = kappa(tables, T1, p1b, lam_um, m_bar, mmr=mmr_fn(i, T1, p1b))
        p1, p2 = p1b * BAR, p2b * BAR
        dtau = (p1 - p2) / g * k
        dtaus.append(dtau)
        omega = sigma / (sigma + k)
        if direction == "emit":
            F2d = F_down[i + 1] if i < nL - 1 else F_toa
        else:
            F2d = F_down[i + 1]
        F1u = F_up[i]
        F2u, F1d = propagate_fluxes(lam_cm, F1u, F2d, T1, T2, dtau, omega, 0.0)
        if err is not None:
            e2d = err["down"][i + 1] if (direction == "absorb" or i < nL - 1) else 0.0
            eu, ed = propagate_error_bound(lam_cm, F1u, F2d, T1, T2, dtau, omega,
                                           err["up"][i], e2d, err["delta"])
            if direction == "absorb" or i < nL - 1:
                err["up"][i + 1] = eu
            err["down"][i] = ed
        if direction == "absorb" or i < nL - 1:
            F_up[i + 1] = F2u
        F_down[i] = F1d
        if bol_fn is None:
            Fb = (trapz(F2u, lam_cm), trapz(F2d, lam_cm), trapz(F1u, lam_cm), trapz(F1d, lam_cm))
        else:  # sharded runs: caller combines slice partial sums (tests/test_distributed_cpu.py)
            Fb = bol_fn(F2u, F2d, F1u, F1d)
        dT[i] = layer_dT(Fb, T1, T2, p1, p2, g, m_bar, alpha)
    return F_up, F_down, T - dT, np.array(dtaus), dT


class ChemistryTable:
    """Mass mixing ratios on (T, p) nodes, values[S][n_T][n_p], T (K) and p (bar) ascending:
    the checker of the engine's frei_set_chemistry interface (no reference counterpart: the
    reference calls FastChem, chemistry.py:114-205, at every kappa; parity against FastChem is
    unpinned).  Linear in T and in log10 p (p in dyn cm^-2, as the engine receives it),
    clamped to the nodes, in the engine's exact operation order
    ((v00 (1 - z) + v01 z) (1 - y) + (v10 (1 - z) + v11 z) y)."""

    def __init__(self, values, T_nodes, p_nodes_bar):
        self.values = np.asarray(values, dtype=float)
        self.T = np.asarray(T_nodes, dtype=float)
        self.logp = np.log10(np.asarray(p_nodes_bar, dtype=float) * BAR)

    @staticmethod
    def _bracket(g, x):
        if g.size < 2:
            return 0, 0.0
        xc = min(max(x, g[0]), g[-1])
        i = int(min(np.searchsorted(g, xc, side="right") - 1, g.size - 2))
        return i, (xc - g[i]) / (g[i + 1] - g[i])

    def __call__(self, T, p_bar):
        it, y = self._bracket(self.T, float(T))
        j, z = self._bracket(self.logp, float(np.log10(p_bar * BAR)))
        out = np.empty(self.values.shape[0])
        for s in range(out.size):
            def row(k):
                r = self.values[s, k]
                return r[j] * (1.0 - z) + r[j + 1] * z if r.size > 1 else r[0]
            a = row(it)
            out[s] = a * (1.0 - y) + row(it + 1) * y if self.T.size > 1 else a
        return out


def _mmr_fn(tables, m_bar, mmr):
    """mmr of every species at layer i, temperature T, pressure p (bar): the mock, a fixed
    [S][n_layers] array, or a ChemistryTable evaluated at (T, p) (opacity.py:246-248)."""
    names = list(tables)
    if mmr is None:
        m = mock_mmr(names, m_bar)
        return lambda i, T, p: m
    if callable(mmr):
        return lambda i, T, p: mmr(T, p)
    mmr = np.asarray(mmr, dtype=float)
    return lambda i, T, p: mmr[:, i]


def emit(tables, T, p_bar, lam_um, F_toa, g, m_bar, alpha=1, fluxes_up=None,
         fluxes_down=None, mmr=None, err=None, bol_fn=None):
    """twostream.py:290-421 with n_timesteps=1 -> (F_up, F_down, T_new, dtaus, dT)."""
    T = np.asarray(T, dtype=float)
    nL, nlam = len(p_bar), len(lam_um)
    F_up = np.zeros((nL, nlam)) if fluxes_up is None else fluxes_up
    if fluxes_down is None:
        F_down = np.zeros((nL, nlam))
        F_down[-1] = F_toa
    else:
        F_down = fluxes_down
    return _sweep("emit", tables, T, np.asarray(p_bar), np.asarray(lam_um), F_toa, g, m_bar,
                  alpha, F_up, F_down, _mmr_fn(tables, m_bar, mmr), err, bol_fn)


def absorb(tables, T, p_bar, lam_um, F_toa, g, m_bar, alpha=1, fluxes_up=None,
           fluxes_down=None, mmr=None, err=None, bol_fn=None):
    """twostream.py:424-550 with n_timesteps=1.  fluxes_up=None -> F_up[0] = pi B(T0) (Q5)."""
    T = np.asarray(T, dtype=float)
    nL, nlam = len(p_bar), len(lam_um)
    if fluxes_up is None:
        F_up = np.zeros((nL, nlam))
        F_up[0] = np.pi * BB(T[0], np.asarray(lam_um) * 1e-4)
    else:
        F_up = fluxes_up
    if fluxes_down is None:
        F_down = np.zeros((nL, nlam))
        F_down[-1] = F_toa
    else:
        F_down = fluxes_down
    return _sweep("absorb", tables, T, np.asarray(p_bar), np.asarray(lam_um), F_toa, g, m_bar,
                  alpha, F_up, F_down, _mmr_fn(tables, m_bar, mmr), err, bol_fn)


def converged(temp_hists, dT_absorb, n_zero_crossings, convergence_dT):
    """core.py:301-318 (Q13)."""
    th = np.hstack(temp_hists)
    th = th.T[th[0] != 0].T
    diffs = np.diff(th.T, axis=0)
    conv = (np.count_nonzero(np.sign(diffs[1:]) != np.sign(diffs[:-1]), axis=0)
            > n_zero_crossings) | (np.abs(dT_absorb) < convergence_dT)
    return bool(np.all(conv))


def emission_spectrum(tables, T_init, p_bar, lam_um, F_toa, g, m_bar, alpha=1,
                      n_timesteps=1, n_zero_crossings=2, convergence_dT=3.0, mmr=None,
                      record=None, err=None, bol_fn=None):
    """core.py:233-338 -> (spectrum, final_T, temp_hist, dtaus, F_up, F_down, n_iter)."""
    nL, nlam = len(p_bar), len(lam_um)
    F_up = np.zeros((nL, nlam))
    F_down = np.zeros((nL, nlam))
    T = np.asarray(T_init, dtype=float).copy()
    hists = []
    it = 0
    for it in range(n_timesteps):
        F_up, F_down, T, _, dTe = emit(tables, T, p_bar, lam_um, F_toa, g, m_bar, alpha,
                                       F_up, F_down, mmr, err, bol_fn)
        if record is not None:
            record.append(("emit", F_up.copy(), F_down.copy(), dTe.copy()))
        T_before = T.copy()
        F_up, F_down, T, _, dTa = absorb(tables, T, p_bar, lam_um, F_toa, g, m_bar, alpha,
                                         F_up, F_down, mmr, err, bol_fn)
        if record is not None:
            record.append(("absorb", F_up.copy(), F_down.copy(), dTa.copy()))
        hists.append(np.stack([T_before, T], axis=1))
        if converged(hists, dTa, n_zero_crossings, convergence_dT):
            break
    th = np.hstack(hists)
    th = th.T[th[0] != 0].T
    # final emit without alpha -> alpha = 1 (Q7)
    F_up, F_down, T, dtaus, _ = emit(tables, T, p_bar, lam_um, F_toa, g, m_bar, 1,
                                     F_up, F_down, mmr, err, bol_fn)
    return F_up[-1].copy(), T, th, dtaus, F_up, F_down, it + 1


# ----------------------------------------------------------------- fixtures
def example_opacity_row(lam_um, seed=42, scale_factor=20):
    """load_example_opacity's per-(p,T) row (opacity.py:272-342); identical at every node."""
    lam = np.asarray(lam_um, dtype=float)
    np.random.seed(seed)
    so = (np.exp(-0.5 * (lam - 6) ** 2 / 2 ** 2) +
          0.8 * np.exp(-0.5 * (lam - 0.3) ** 2 / 0.5 ** 2))
    for amp, wl in zip(np.random.uniform(low=0.1, high=0.2, size=15),
                       np.random.uniform(low=0.5, high=1, size=15)):
        so += amp * np.exp(-0.5 * (lam - wl) ** 2 / 0.005 ** 2)
    for amp, wl in zip([0.22, 0.2, 0.18], np.logspace(np.log10(1.4), np.log10(2.7), 3)):
        so += amp * np.exp(-0.5 * (lam - wl) ** 2 / 0.13 ** 2)
    row = np.zeros(lam.size)
    row += 5 * 10 ** (2.5 * (so - 0.4))
    return row * scale_factor


def example_opacity(p_bar, T_nodes, lam_um, seed=42, scale_factor=20):
    row = example_opacity_row(lam_um, seed, scale_factor)
    _, idx = np.unique(T_nodes, return_index=True)   # drop_duplicates('temperature')
    Tn = np.asarray(T_nodes)[np.sort(idx)]
    vals = np.broadcast_to(row, (len(p_bar), len(Tn), row.size))
    return {"1H2-16O": Table(vals, p_bar, Tn, lam_um)}


def separable_table(base, fp, fT, lo=1e-4, hi=1e3):
    """Synthetic separable table used by the goldens/bench: clip(fp[p]*fT[T]*base[lam])."""
    return np.clip((fp[:, None] * fT[None, :])[:, :, None] * base[None, None, :], lo, hi)


class SeparableValues:
    """Lazy (n_p, n_T, n_lam) view of separable_table(base, fp, fT): rows are built on
    indexing, so the CPU baseline can run large grids without materialising the table."""

    def __init__(self, base, fp, fT, lo=1e-4, hi=1e3):
        self.base, self.fp, self.fT = (np.asarray(a, dtype=float) for a in (base, fp, fT))
        self.lo, self.hi = lo, hi
        self.shape = (self.fp.size, self.fT.size, self.base.size)

    def __getitem__(self, pidx):
        fp = self.fp[pidx]
        return np.clip((fp[:, None] * self.fT[None, :])[:, :, None] * self.base[None, None, :],
                       self.lo, self.hi)

    def row(self, pi, ti):
        """self[pi][ti]: clip((fp[pi] fT[ti]) base) — the same operations in the same order."""
        return np.clip((self.fp[pi] * self.fT[ti]) * self.base, self.lo, self.hi)


# ----------------------------------------------------------------- opacity binning (§8(f) #1)
# binned_opacity (opacity.py:66-170): high-resolution cross-sections in the
# opacity_dir_to_netcdf layout (opacity.py:395-483: float32 (temperature, pressure,
# wavelength), wavelength µm ascending) binned onto a Grid's wavelength bins, then the
# nearest source (T, p) node is taken for every target node.  Pinned by
# tests/golden/binning.npz (the reference's own binned_opacity + interp.py, run under
# tests/golden/binharness.py stand-ins for numba/numpy_groupies/xarray; real pandas).
def nearest_index(nodes, targets):
    """xarray interp(method='nearest', fill_value='extrapolate') index selection: sortby,
    then scipy interp1d 'nearest' — midpoints x[i]/2 + x[i+1]/2, searchsorted side='left'
    (a target exactly on a midpoint takes the lower node), clipped to the end nodes."""
    nodes = np.asarray(nodes, dtype=float)
    order = np.argsort(nodes, kind="stable")
    x = nodes[order]
    if x.size == 1:
        return np.zeros(np.size(targets), dtype=np.int64) + order[0]
    h = x / 2.0
    bds = h[1:] + h[:-1]
    idx = np.clip(np.searchsorted(bds, np.asarray(targets, dtype=float), side="left"),
                  0, x.size - 1)
    return order[idx]


def bin_ranges(wl_hi, wl_bins):
    """pandas.cut(right=True) bin membership on the cropped axis
    wl_bins.min() < x < wl_bins.max() (opacity.py:131-135, interp.py:289): point ranges
    [start_k, end_k) of bin k = (b_k, b_{k+1}] for an ascending high-res axis."""
    wl_hi = np.asarray(wl_hi, dtype=float)
    b = np.asarray(wl_bins, dtype=float)
    if np.any(np.diff(wl_hi) <= 0) or np.any(np.diff(b) <= 0):
        raise ValueError("wavelengths and bin edges must be strictly ascending")
    start = np.searchsorted(wl_hi, b[:-1], side="right")
    end = np.searchsorted(wl_hi, b[1:], side="right")
    end[-1] = np.searchsorted(wl_hi, b[-1], side="left")   # x < wl_bins.max() (cropping)
    return start.astype(np.int64), np.maximum(end, start).astype(np.int64)


def bin_groupies_rows(rows_f32, start, end, wl_bins):
    """groupby_bins_agg(..., func=np.trapz) * (wl_bins[1:] - wl_bins[:-1]) * 1e-3
    (opacity.py:136-139; interp.py:156-207, 246-307).  Per row and bin: the pair rule of
    AggregateTrapz._loop — consecutive points i, i+1 in the same bin add
    ((a_i + a_{i+1}) / 2) * dx with dx = 1 (_binned_agg passes no x) — into a float32
    accumulator (numpy_groupies check_dtype keeps the input dtype; numba forms
    f32(a_i + a_{i+1}) / 2 in float64 and rounds the sum to float32 on every +=).
    Sequential in point order.  Bins with < 2 points stay 0 (fill_value)."""
    rows = np.asarray(rows_f32, dtype=np.float32).reshape(-1, rows_f32.shape[-1])
    n = end - start
    acc = np.zeros((rows.shape[0], start.size), dtype=np.float32)
    for j in range(int(n.max()) - 1 if n.size else 0):
        m = j + 1 < n
        i = start[m] + j
        pair = rows[:, i] + rows[:, i + 1]                       # float32 add
        acc[:, m] = (acc[:, m].astype(np.float64) + pair.astype(np.float64) / 2
                     ).astype(np.float32)
    out = acc.astype(np.float64) * (np.asarray(wl_bins)[1:] - np.asarray(wl_bins)[:-1]) * 1e-3
    return out.reshape(rows_f32.shape[:-1] + (start.size,))


def bin_exact_groups(wl_hi, start, end):
    """Non-empty groups of xarray groupby_bins (empty bins dropped, opacity.py:156) and
    their coordinates wl.mean() (opacity.py:42)."""
    keep = end > start
    gs, ge = start[keep], end[keep]
    centres = np.array([np.mean(wl_hi[s:e]) for s, e in zip(gs, ge)])
    return gs, ge, centres


def bin_exact_rows(rows_f32, wl_hi, start, end, lam_um):
    """mapfunc_exact + interp onto lam (opacity.py:33-42, 155-167): per non-empty bin,
    integrate('wavelength') (xarray trapz: dx * 0.5 * (y[1:] + y[:-1]), float32 pair sum,
    float64 integrand, summed in point order) / (wl.max() - wl.min()) — a single-point
    bin gives 0/0 = NaN — at coordinate wl.mean(); then scipy interp1d linear with
    fill_value='extrapolate' onto lam: slope = (y_hi - y_lo) / (x_hi - x_lo),
    y = slope * (x - x_lo) + y_lo, interval = clip(searchsorted(x, lam), 1, n - 1)."""
    rows = np.asarray(rows_f32, dtype=np.float32).reshape(-1, rows_f32.shape[-1])
    wl_hi = np.asarray(wl_hi, dtype=float)
    gs, ge, x = bin_exact_groups(wl_hi, start, end)
    if x.size < 2:
        raise ValueError("x and y arrays must have at least 2 entries")
    y = np.zeros((rows.shape[0], x.size))
    n = ge - gs
    with np.errstate(invalid="ignore", divide="ignore"):
        for j in range(int(n.max()) - 1):        # point order within every group
            m = j + 1 < n
            i = gs[m] + j
            integrand = (wl_hi[i + 1] - wl_hi[i]) * 0.5 * (rows[:, i + 1] + rows[:, i])
            y[:, m] = y[:, m] + integrand
        y = y / (wl_hi[ge - 1] - wl_hi[gs])
        lam = np.asarray(lam_um, dtype=float)
        hi = np.clip(np.searchsorted(x, lam), 1, x.size - 1)
        lo = hi - 1
        slope = (y[:, hi] - y[:, lo]) / (x[hi] - x[lo])
        out = slope * (lam - x[lo]) + y[:, lo]
    return out.reshape(rows_f32.shape[:-1] + (lam.size,))


def binned_opacity(xsec, xsec_T, xsec_p, wl_hi, temperatures, pressures_bar, wl_bins, lam_um,
                   groupies=True):
    """One species of binned_opacity (opacity.py:66-170) -> (pressure, temperature, λ)
    table (this oracle's Table layout; the reference's DataArray is (temperature,
    pressure, wavelength) for groupies and (wavelength, temperature, pressure) for the
    exact path)."""
    start, end = bin_ranges(wl_hi, wl_bins)
    ti = nearest_index(xsec_T, temperatures)
    pi = nearest_index(xsec_p, pressures_bar)
    # bin only the source rows the nearest selection uses (selection commutes with binning)
    pairs = sorted({(a, b) for a in ti for b in pi})
    rows = np.stack([xsec[a, b] for a, b in pairs])
    binned = (bin_groupies_rows(rows, start, end, wl_bins) if groupies
              else bin_exact_rows(rows, wl_hi, start, end, lam_um))
    where = {pq: k for k, pq in enumerate(pairs)}
    out = np.empty((len(pi), len(ti), binned.shape[-1]))
    for kp, b in enumerate(pi):
        for kt, a in enumerate(ti):
            out[kp, kt] = binned[where[(a, b)]]
    return out


# ----------------------------------------------------------------- post-processing (§8(f) #3)
# Pinned by tests/golden/post_c1.npz (the reference's effective_temperature and dashboard
# contribution function on a converged C1 atmosphere).
def milne_pressures(dtaus, p_bar):
    """Per-wavelength Milne pressure (core.py:392-395): np.interp(2/3, exp(-dtaus[:, i]),
    pressures) — numpy's interp on the (unsorted) per-layer transmissions."""
    dtaus = np.asarray(dtaus, dtype=float)
    return np.array([np.interp(2 / 3, np.exp(-dtaus[:, i]), p_bar)
                     for i in range(dtaus.shape[1])])


def effective_temperature_milne(lam_um, p_bar, spectrum, dtaus, final_T):
    """core.py:386-405: weights = F_lambda -> erg s^-1 cm^-2 (astropy spectral_density:
    lambda F_lambda), then interp of the weighted mean pressure on the reversed T-P
    profile."""
    pm = milne_pressures(dtaus, p_bar)
    w = np.asarray(spectrum) * (np.asarray(lam_um) * 1e-4)
    return np.interp(np.average(pm, weights=w), np.asarray(p_bar)[::-1],
                     np.asarray(final_T)[::-1])


def effective_temperature_planck(lam_um, spectrum):
    """core.py:408-414: (trapz(F, lam) / sigma_SB) ** (1/4), lam in cm."""
    lam_cm = np.asarray(lam_um) * 1e-4
    f = np.asarray(spectrum)
    bol = np.sum(np.diff(lam_cm) * (f[1:] + f[:-1]) / 2.0)
    return (bol / SIGMA_SB) ** 0.25


def effective_temperature(lam_um, p_bar, spectrum, dtaus, final_T):
    """core.py:417-439: mean of the Milne and Stefan-Boltzmann estimates."""
    return float(np.mean([effective_temperature_milne(lam_um, p_bar, spectrum, dtaus, final_T),
                          effective_temperature_planck(lam_um, spectrum)]))


def contribution_function(lam_um, p_bar, final_T, dtaus):
    """dashboard's contribution function (plot.py:63-79) in cgs, returned as plotted
    (cf[::-1]: rows bottom-first like the pressures):
    tau = cumsum(dtaus[::-1]); cf = exp(-tau) * dtau * (p / dP) * nu^3 / expm1(hc nu / k T),
    normalised over layers at every wavelength."""
    dtaus = np.asarray(dtaus, dtype=float)
    p = np.asarray(p_bar, dtype=float)
    tau = np.cumsum(dtaus[::-1], axis=0)
    nus = 1.0 / (np.asarray(lam_um) * 1e-4)
    hcperk = H * C / K_B
    dlogP = (np.log10(p.max()) - np.log10(p.min())) / (len(p) - 1)
    k = 10 ** -dlogP
    dParr = (1 - k) * p
    T = np.asarray(final_T, dtype=float)
    with np.errstate(invalid="ignore", divide="ignore"):
        cf = (np.exp(-tau) * dtaus[::-1] * (p[::-1, None] / dParr[::-1, None]) *
              nus ** 3 / np.expm1(hcperk * nus / T[::-1, None]))
        cf /= np.sum(cf, axis=0)
    return cf[::-1]
