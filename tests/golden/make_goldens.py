"""Generate golden vectors from the reference implementation (build container only).

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 -W ignore tests/golden/make_goldens.py

Imports the read-only reference through ``refharness`` (stand-ins per SURVEY.md
Appendix B), runs its hot-path functions on fixed inputs and writes plain
``.npz`` arrays (inputs + outputs, no pickles) next to this script.  Units in
the fixtures: wavelength µm, pressure bar, temperature K, flux erg s^-1 cm^-3,
opacity cm^2 g^-1, g cm s^-2, masses g.

Cases (file -> reference functions exercised):
  setup_c1.npz      Grid/Planet/F_TOA/wavelength_grid/pressure_grid/temperature_grid,
                    load_example_opacity row, mock chemistry mmr   (core.py:34-188, tp.py, opacity.py:272-342, chemistry.py:114-246)
  propagate.npz     propagate_fluxes on random vectors incl. omega_0>0.1, tiny dtau, T1==T2  (twostream.py:97-177)
  kappa.npz         kappa: on/off-node T, outside hull, off-node p, 2-species T-varying table,
                    single-T (1-D) table   (opacity.py:203-269)
  emit_absorb_c1.npz  standalone emit / absorb with fluxes=None   (twostream.py:290-550)
  c1_step1.npz      Grid.emission_spectrum(n_timesteps=1), example opacity + gray variant (core.py:233-338)
  c1_converge.npz   Grid.emission_spectrum(n_timesteps=100) to convergence
  c2small.npz       60 x 2048, 2 species separable T-varying tables (16 T nodes), 3 iterations
  c2strong.npz      c2small's grid and line forests at 1e3x strength, clipped to [10, 1e3]
                    cm^2 g^-1: a well-conditioned twin (the reference algorithm's one-ulp floor
                    3e-13, against c2small's 2.4e-10), held to 1e-10 outright (round 6)
  c1_vmr3e4.npz     test_core.py:19-71's Grid (example opacity, n_timesteps=1) with kappa's
                    chemistry a constant VMR of 3e-4 -- the H2O maximum FastChem gives in the
                    reference's CI (test_chemistry.py:45-46), which reproduces its pins
                    (test_core.py:51-71)   (opacity.py:246-248, core.py:233-338)
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refharness as H  # noqa: E402

import numpy as np  # noqa: E402
import astropy.units as u  # noqa: E402

R = H.load()
FLUX = u.erg / u.s / u.cm ** 3
KAP = u.cm ** 2 / u.g


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
    print(f"wrote {name}: {os.path.getsize(path) / 1024:.1f} KiB")


def planet():
    return R.core.Planet.from_hot_jupiter()


def planet_arrays(pl):
    return dict(g=pl.g.to(u.cm / u.s ** 2).value, m_bar=pl.m_bar.to(u.g).value,
                a_rstar=pl.a_rstar, T_star=pl.T_star.to(u.K).value, alpha=pl.alpha)


def grid_arrays(g):
    return dict(lam=g.lam.to(u.um).value, wl_bins=np.asarray(g.wl_bins), R=g.R,
                pressures=g.pressures.to(u.bar).value,
                init_temperatures=g.init_temperatures.to(u.K).value)


# ---------------------------------------------------------------- recorders
class Recorder:
    """Wraps core.emit / core.absorb to record every sweep inside emission_spectrum."""

    def __init__(self):
        self.calls = []
        self._emit, self._absorb = R.core.emit, R.core.absorb

    def __enter__(self):
        def wrap(fn, kind):
            def inner(*a, **kw):
                T_in = kw["temperatures"].to(u.K).value.copy()
                out = fn(*a, **kw)
                fu, fd, Tf, Th, dtaus, dT = out
                self.calls.append(dict(kind=kind, T_in=T_in, T_out=Tf.to(u.K).value.copy(),
                                       dT=dT.to(u.K).value.copy(),
                                       F_up=fu.to(FLUX).value.copy(),
                                       F_down=fd.to(FLUX).value.copy(),
                                       dtaus=np.asarray(dtaus, dtype=float)))
                return out
            return inner
        R.core.emit = wrap(self._emit, "emit")
        R.core.absorb = wrap(self._absorb, "absorb")
        return self

    def __exit__(self, *exc):
        R.core.emit, R.core.absorb = self._emit, self._absorb


def spectrum_case(grid, n_timesteps, prefix, **kw):
    with Recorder() as rec:
        t0 = time.time()
        spec, T, th, dtaus = grid.emission_spectrum(n_timesteps=n_timesteps, **kw)
        wall = time.time() - t0
    last = rec.calls[-1]
    out = {
        prefix + "spectrum": spec.flux.to(FLUX).value,
        prefix + "final_T": T.to(u.K).value,
        prefix + "temp_hist": th.to(u.K).value,
        prefix + "dtaus": np.asarray(dtaus, dtype=float),
        prefix + "F_up": last["F_up"], prefix + "F_down": last["F_down"],
        prefix + "n_sweeps": len(rec.calls), prefix + "wall_s": wall,
        # per-sweep temperatures (input to each sweep) and dT
        prefix + "sweep_T_in": np.array([c["T_in"] for c in rec.calls]),
        prefix + "sweep_dT": np.array([c["dT"] for c in rec.calls]),
    }
    # fluxes after the first emit and first absorb (interior-row parity)
    out[prefix + "F_up_sweep0"] = rec.calls[0]["F_up"]
    out[prefix + "F_down_sweep0"] = rec.calls[0]["F_down"]
    if len(rec.calls) > 1:
        out[prefix + "F_up_sweep1"] = rec.calls[1]["F_up"]
        out[prefix + "F_down_sweep1"] = rec.calls[1]["F_down"]
    return out, spec, T, dtaus


# ---------------------------------------------------------------- cases
def case_setup():
    pl = planet()
    g = R.core.Grid(pl, T_ref=2400 * u.K)
    F_toa = R.core.F_TOA(g.lam, T_star=pl.T_star, a_rstar=pl.a_rstar)
    ex1 = R.opacity.load_example_opacity(g, scale_factor=1)["1H2-16O"]
    ex20 = R.opacity.load_example_opacity(g)["1H2-16O"]
    sig = (R.opacity.rayleigh_H2(g.lam, pl.m_bar) + R.opacity.rayleigh_He(g.lam, pl.m_bar))
    species = ["1H2-16O", "12C-16O", "12C-16O2", "12C-1H4", "Na", "K"]
    mmr = R.chemistry.chemistry(g.init_temperatures, g.pressures, species, m_bar=pl.m_bar)
    # a second, non-default grid (explicit args)
    g2 = R.core.Grid(pl, n_wl_bins=300, n_layers=15, T_ref=2400 * u.K,
                     lam_min=0.7 * u.um, lam_max=5 * u.um, P_toa=1e-5 * u.bar,
                     P_boa=100 * u.bar, P_ref=0.2 * u.bar, alpha=0.12)
    save("setup_c1.npz", **planet_arrays(pl), **grid_arrays(g),
         F_TOA=F_toa.to(FLUX).value,
         example_row_scale1=ex1.values[0, 0], example_row_scale20=ex20.values[0, 0],
         example_shape=np.array(ex1.values.shape),
         example_temperature=ex1.temperature, example_pressure=ex1.pressure,
         example_identical=np.array(bool(np.all(ex1.values == ex1.values[0, 0]))),
         sigma_SI=sig.to(u.m ** 2 / u.kg).value, sigma_cgs=sig.to(KAP).value,
         species=np.array(species), mmr=np.array([mmr[s] for s in species]),
         g2_lam=g2.lam.to(u.um).value, g2_wl_bins=np.asarray(g2.wl_bins), g2_R=g2.R,
         g2_pressures=g2.pressures.to(u.bar).value,
         g2_init_temperatures=g2.init_temperatures.to(u.K).value)


def case_propagate():
    rng = np.random.default_rng(1234)
    n = 1024
    lam = np.logspace(np.log10(0.5), np.log10(10), n) * u.um
    cases = [(2000.0, 1900.0), (800.0, 780.0), (1500.0, 1500.0), (3000.0, 3300.0)]
    out = dict(lam=lam.value)
    for c, (T1, T2) in enumerate(cases):
        dtau = 10 ** rng.uniform(-7, 3, n)
        omega = rng.uniform(0.0, 0.49, n)
        F1u = 10 ** rng.uniform(8, 13, n) * FLUX
        F2d = 10 ** rng.uniform(6, 12, n) * FLUX
        F2u, F1d = R.twostream.propagate_fluxes(lam, F1u, F2d, T1 * u.K, T2 * u.K,
                                                dtau, omega_0=omega, g_0=0)
        out.update({f"c{c}_T1": T1, f"c{c}_T2": T2, f"c{c}_dtau": dtau,
                    f"c{c}_omega": omega, f"c{c}_F1u": F1u.value, f"c{c}_F2d": F2d.value,
                    f"c{c}_F2u": F2u.to(FLUX).value, f"c{c}_F1d": F1d.to(FLUX).value})
    out["n_cases"] = len(cases)
    save("propagate.npz", **out)


def case_propagate_g0():
    """propagate_fluxes with a nonzero asymmetry factor g_0 (twostream.py:139-176): array
    g_0 of both signs, a scalar g_0, omega_0 on both sides of E's 0.1 branch."""
    rng = np.random.default_rng(4321)
    n = 1024
    lam = np.logspace(np.log10(0.5), np.log10(10), n) * u.um
    cases = [(2000.0, 1900.0, "array"), (800.0, 780.0, "array"), (1500.0, 1500.0, 0.35),
             (3000.0, 3300.0, -0.2)]
    out = dict(lam=lam.value)
    for c, (T1, T2, g0) in enumerate(cases):
        dtau = 10 ** rng.uniform(-7, 3, n)
        omega = rng.uniform(0.0, 0.95, n)
        g = rng.uniform(-0.9, 0.9, n) if isinstance(g0, str) else np.float64(g0)
        F1u = 10 ** rng.uniform(8, 13, n) * FLUX
        F2d = 10 ** rng.uniform(6, 12, n) * FLUX
        F2u, F1d = R.twostream.propagate_fluxes(lam, F1u, F2d, T1 * u.K, T2 * u.K,
                                                dtau, omega_0=omega, g_0=g)
        out.update({f"c{c}_T1": T1, f"c{c}_T2": T2, f"c{c}_dtau": dtau,
                    f"c{c}_omega": omega, f"c{c}_g0": g, f"c{c}_F1u": F1u.value,
                    f"c{c}_F2d": F2d.value, f"c{c}_F2u": F2u.to(FLUX).value,
                    f"c{c}_F1d": F1d.to(FLUX).value})
    out["n_cases"] = len(cases)
    save("propagate_g0.npz", **out)


def separable_table(rng, lam_um, p_bar, T_nodes, lo=1e-4, hi=1e3, n_lines=200):
    """Synthetic log-normal line forest (SURVEY.md §8(d) C2 recipe), separable in (p, T)."""
    n = lam_um.size
    x = np.log(lam_um)
    logk = -1.0 + 0.8 * np.sin(2.1 * x) + 0.3 * np.cos(5.3 * x)
    centres = rng.integers(0, n, n_lines)
    strengths = rng.lognormal(0.0, 1.0, n_lines)
    k = np.arange(n)
    for c0, s0 in zip(centres, strengths):
        logk = logk + s0 * np.exp(-0.5 * ((k - c0) / 2.0) ** 2)
    base = 10 ** logk
    fT = (T_nodes / 1000.0) ** 0.5
    fp = (p_bar / 1.0) ** 0.1
    return base, fp, fT


def build_table(base, fp, fT, lo=1e-4, hi=1e3):
    return np.clip((fp[:, None] * fT[None, :])[:, :, None] * base[None, None, :], lo, hi)


def case_kappa():
    pl = planet()
    g = R.core.Grid(pl, T_ref=2400 * u.K)
    op = R.opacity.load_example_opacity(g, scale_factor=1)
    T0, p0 = g.init_temperatures, g.pressures
    Tn = np.sort(op["1H2-16O"].temperature)
    pts = [  # (T K, p bar)
        (T0[0].value, p0[0].value),                      # test_core.py:33-38 call
        (T0[5].value, p0[5].value),                      # on-node T (also a node of p)
        (0.5 * (Tn[3] + Tn[4]), p0[7].value),            # off-node T
        (Tn[-1] + 50.0, p0[2].value),                    # above the hull -> fill 0
        (Tn[0] - 1.0, p0[-1].value),                     # below the hull -> fill 0
        (Tn[0], p0[-1].value),                           # exactly the min node
        (Tn[-1], p0[0].value),                           # exactly the max node
        (0.3 * Tn[2] + 0.7 * Tn[3], np.sqrt(p0[10].value * p0[11].value)),  # off-node p
    ]
    out = dict(ex_T=np.array([p[0] for p in pts]), ex_p=np.array([p[1] for p in pts]))
    ks, ss = [], []
    for T, p in pts:
        k, s = R.opacity.kappa(op, T * u.K, p * u.bar, g.lam, m_bar=pl.m_bar)
        ks.append(k.to(KAP).value)
        ss.append(s.to(KAP).value)
    out.update(ex_k=np.array(ks), ex_sigma=np.array(ss))

    # 2-species T-varying separable tables on a small grid
    gs = R.core.Grid(pl, n_wl_bins=256, n_layers=12, T_ref=1500 * u.K)
    lam = gs.lam.to(u.um).value
    pb = gs.pressures.to(u.bar).value
    Tmin, Tmax = gs.init_temperatures.value.min(), gs.init_temperatures.value.max()
    T_nodes = np.linspace(0.8 * Tmin, 1.2 * Tmax, 9)
    rng = np.random.default_rng(7)
    tabs = {}
    for s, name in enumerate(["1H2-16O", "12C-16O"]):
        base, fp, fT = separable_table(rng, lam, pb, T_nodes, n_lines=60)
        out[f"sep{s}_base"], out[f"sep{s}_fp"], out[f"sep{s}_fT"] = base, fp, fT
        tabs[name] = R.DataArray(build_table(base, fp, fT),
                                 dims=["pressure", "temperature", "wavelength"],
                                 coords=dict(pressure=pb, temperature=T_nodes, wavelength=lam))
    pts2 = [(gs.init_temperatures[i].value, pb[i]) for i in range(12)]
    pts2 += [(T_nodes[0] - 5, pb[3]), (T_nodes[-1] + 5, pb[3]), (T_nodes[4], pb[6]),
             (0.5 * (T_nodes[2] + T_nodes[3]), np.sqrt(pb[4] * pb[5]))]
    ks, ss = [], []
    for T, p in pts2:
        k, s = R.opacity.kappa(tabs, T * u.K, p * u.bar, gs.lam, m_bar=pl.m_bar)
        ks.append(k.to(KAP).value)
        ss.append(s.to(KAP).value)
    out.update(sep_lam=lam, sep_p=pb, sep_Tnodes=T_nodes,
               sep_T=np.array([p[0] for p in pts2]), sep_pq=np.array([p[1] for p in pts2]),
               sep_k=np.array(ks), sep_sigma=np.array(ss))

    # single-T (1-D, pressure-only) table: every row scaled by fp only
    base, fp, _ = separable_table(np.random.default_rng(9), lam, pb, T_nodes[:1], n_lines=30)
    one = R.DataArray(np.clip(fp[:, None, None] * base[None, None, :], 1e-4, 1e3),
                      dims=["pressure", "temperature", "wavelength"],
                      coords=dict(pressure=pb, temperature=[1234.0], wavelength=lam))
    pts3 = [(1000.0, pb[2]), (2500.0, pb[5]), (1500.0, np.sqrt(pb[7] * pb[8])), (1500.0, pb[-1])]
    ks = []
    for T, p in pts3:
        k, s = R.opacity.kappa({"1H2-16O": one}, T * u.K, p * u.bar, gs.lam, m_bar=pl.m_bar)
        ks.append(k.to(KAP).value)
    out.update(oneT_base=base, oneT_fp=fp, oneT_T=np.array([p[0] for p in pts3]),
               oneT_p=np.array([p[1] for p in pts3]), oneT_k=np.array(ks))
    save("kappa.npz", **out)


def case_emit_absorb():
    pl = planet()
    g = R.core.Grid(pl, T_ref=2400 * u.K)
    op = R.opacity.load_example_opacity(g, scale_factor=1)
    F_toa = R.core.F_TOA(g.lam, T_star=pl.T_star, a_rstar=pl.a_rstar)
    out = {}
    for kind, fn in (("emit", R.twostream.emit), ("absorb", R.twostream.absorb)):
        fu, fd, Tf, Th, dtaus, dT = fn(op, g.init_temperatures, g.pressures, g.lam, F_toa,
                                      pl.g, m_bar=pl.m_bar, n_timesteps=1, alpha=1)
        out.update({f"{kind}_F_up": fu.to(FLUX).value, f"{kind}_F_down": fd.to(FLUX).value,
                    f"{kind}_T": Tf.to(u.K).value, f"{kind}_dtaus": np.asarray(dtaus, float),
                    f"{kind}_dT": dT.to(u.K).value})
    save("emit_absorb_c1.npz", **out)


def case_c1_step1():
    pl = planet()
    g = R.core.Grid(pl, T_ref=2400 * u.K)
    g.load_opacities(opacities=R.opacity.load_example_opacity(g, scale_factor=1))
    out, spec, T, dtaus = spectrum_case(g, 1, "ex_")
    out["ex_Teff"] = R.core.effective_temperature(g, spec, dtaus, T).to(u.K).value
    out["ex_Teff_milne"] = R.core.effective_temperature_milne(g, spec, dtaus, T)
    out["ex_Teff_planck"] = R.core.effective_temperature_planck(g, spec).to(u.K).value
    # gray variant: lambda-constant table kappa = 1 cm^2/g
    gg = R.core.Grid(pl, T_ref=2400 * u.K)
    gray = R.DataArray(np.ones((30, 30, 500)), dims=["pressure", "temperature", "wavelength"],
                       coords=dict(pressure=gg.pressures.to(u.bar).value,
                                   temperature=gg.init_temperatures.value,
                                   wavelength=gg.lam.to(u.um).value))
    gg.load_opacities(opacities={"1H2-16O": gray})
    o2, _, _, _ = spectrum_case(gg, 1, "gray_")
    out.update(o2)
    save("c1_step1.npz", **out)


def case_c1_converge():
    pl = planet()
    g = R.core.Grid(pl, T_ref=2400 * u.K)
    g.load_opacities(opacities=R.opacity.load_example_opacity(g, scale_factor=1))
    out, spec, T, dtaus = spectrum_case(g, 100, "cv_")
    # per-sweep T inputs are enough to replay every iteration; drop per-sweep fluxes
    save("c1_converge.npz", **out)
    print("converged after", out["cv_n_sweeps"], "sweeps in", out["cv_wall_s"], "s")


def case_c2small():
    pl = planet()
    g = R.core.Grid(pl, n_wl_bins=2048, n_layers=60, T_ref=1500 * u.K)
    lam = g.lam.to(u.um).value
    pb = g.pressures.to(u.bar).value
    Tmin, Tmax = g.init_temperatures.value.min(), g.init_temperatures.value.max()
    T_nodes = np.linspace(0.8 * Tmin, 1.2 * Tmax, 16)
    out = dict(lam=lam, pressures=pb, init_temperatures=g.init_temperatures.value,
               T_nodes=T_nodes)
    tabs = {}
    for s, name in enumerate(["1H2-16O", "12C-16O"]):
        base, fp, fT = separable_table(np.random.default_rng(42 + s), lam, pb, T_nodes)
        out[f"s{s}_base"], out[f"s{s}_fp"], out[f"s{s}_fT"] = base, fp, fT
        tabs[name] = R.DataArray(build_table(base, fp, fT),
                                 dims=["pressure", "temperature", "wavelength"],
                                 coords=dict(pressure=pb, temperature=T_nodes, wavelength=lam))
    g.load_opacities(opacities=tabs)
    o, _, _, _ = spectrum_case(g, 3, "")
    out.update(o)
    save("c2small.npz", **out)


def case_c2strong():
    """c2small's Grid and line forests, 1e3 times stronger and clipped to [10, 1e3]: no layer is
    optically thin, so the reference's own one-ulp floor is 3e-13 (c2small: 2.4e-10) and a 1e-10
    comparison needs no floor rule."""
    pl = planet()
    g = R.core.Grid(pl, n_wl_bins=2048, n_layers=60, T_ref=1500 * u.K)
    lam = g.lam.to(u.um).value
    pb = g.pressures.to(u.bar).value
    Tmin, Tmax = g.init_temperatures.value.min(), g.init_temperatures.value.max()
    T_nodes = np.linspace(0.8 * Tmin, 1.2 * Tmax, 16)
    out = dict(lam=lam, pressures=pb, init_temperatures=g.init_temperatures.value,
               T_nodes=T_nodes, clip_lo=10.0, clip_hi=1e3)
    tabs = {}
    for s, name in enumerate(["1H2-16O", "12C-16O"]):
        base, fp, fT = separable_table(np.random.default_rng(42 + s), lam, pb, T_nodes)
        base = base * 1e3
        out[f"s{s}_base"], out[f"s{s}_fp"], out[f"s{s}_fT"] = base, fp, fT
        tabs[name] = R.DataArray(build_table(base, fp, fT, lo=10.0, hi=1e3),
                                 dims=["pressure", "temperature", "wavelength"],
                                 coords=dict(pressure=pb, temperature=T_nodes, wavelength=lam))
    g.load_opacities(opacities=tabs)
    o, _, _, _ = spectrum_case(g, 3, "")
    out.update(o)
    save("c2strong.npz", **out)


def vmr_chemistry(vmr):
    """A chemistry provider on the reference's signature (chemistry.py:114-116) returning a
    constant volume mixing ratio ``vmr`` for every species: mmr = vmr * mass / m_bar, the
    mock's formula (chemistry.py:197-199, 243) with another VMR."""
    def chemistry(temperatures, pressures, species, return_vmr=False, m_bar=None):
        n = np.atleast_1d(temperatures.value).shape
        mmr = {iso: np.full(n, vmr) * (R.chemistry.iso_to_mass(iso) / m_bar)
               .to(u.dimensionless_unscaled).value for iso in species}
        return (mmr, {iso: np.full(n, vmr) for iso in species}) if return_vmr else mmr
    return chemistry


def case_c1_vmr3e4():
    pl = planet()
    g = R.core.Grid(pl, T_ref=2400 * u.K)
    g.load_opacities(opacities=R.opacity.load_example_opacity(g, scale_factor=1))
    chem = vmr_chemistry(3e-4)
    saved = R.opacity.chemistry
    R.opacity.chemistry = chem            # what kappa calls (opacity.py:11, 246-248)
    try:
        out, spec, T, dtaus = spectrum_case(g, 1, "")
        out["Teff"] = R.core.effective_temperature(g, spec, dtaus, T).to(u.K).value
    finally:
        R.opacity.chemistry = saved
    out["lam"] = g.lam.to(u.um).value
    out["peak_lam"] = spec.wavelength[spec.flux.argmax()].to(u.um).value
    out["peak_flux"] = spec.flux.max().to(FLUX).value
    out["mmr"] = chem(g.init_temperatures, g.pressures, ["1H2-16O"], m_bar=pl.m_bar)["1H2-16O"]
    save("c1_vmr3e4.npz", **out)
    print("peak", out["peak_lam"], "um", out["peak_flux"], "Teff", out["Teff"])


if __name__ == "__main__":
    which = sys.argv[1:] or ["setup", "propagate", "kappa", "emit_absorb", "c1_step1",
                             "c2small", "c1_converge"]
    for w in which:
        t0 = time.time()
        globals()["case_" + w]()
        print(f"  case {w}: {time.time() - t0:.1f} s")
