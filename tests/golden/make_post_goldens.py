"""Golden vectors of the reference's post-processing on a converged C1 atmosphere (build
container only):

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 -W ignore tests/golden/make_post_goldens.py

* ``effective_temperature`` and its two parts (core.py:386-439), with the per-wavelength
  Milne pressures recorded from the reference's own ``np.interp`` calls
  (core.py:392-395);
* the contribution function of ``dashboard`` (plot.py:63-79), captured as the array the
  reference hands to ``pcolormesh`` (``cf[::-1]``), Agg backend.
Writes ``post_c1.npz`` (inputs + outputs, no pickles)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refharness as H  # noqa: E402

import matplotlib  # noqa: E402
matplotlib.use("Agg")
import matplotlib.axes  # noqa: E402
import numpy as np  # noqa: E402
import astropy.units as u  # noqa: E402

R = H.load()
import importlib  # noqa: E402
plot = importlib.import_module("frei.plot")
FLUX = u.erg / u.s / u.cm ** 3


def main():
    pl = R.core.Planet.from_hot_jupiter()
    g = R.core.Grid(pl, T_ref=2400 * u.K)
    op = R.opacity.load_example_opacity(g, scale_factor=1)
    g.load_opacities(opacities=op)
    spec, T, th, dtaus = g.emission_spectrum(n_timesteps=100)
    # Milne pressures: the first n_lam np.interp calls of effective_temperature_milne
    calls = []
    orig = np.interp

    def rec(x, xp, fp, *a, **k):
        r = orig(x, xp, fp, *a, **k)
        calls.append(np.asarray(getattr(r, "value", r), dtype=float).copy())
        return r
    np.interp = rec
    try:
        t_milne = R.core.effective_temperature_milne(g, spec, dtaus, T)
    finally:
        np.interp = orig
    p_milne = np.array([float(c) for c in calls[:g.lam.size]])
    t_planck = R.core.effective_temperature_planck(g, spec)
    t_eff = R.core.effective_temperature(g, spec, dtaus, T)
    # contribution function: the array dashboard passes to pcolormesh
    got = {}
    orig_pm = matplotlib.axes.Axes.pcolormesh

    def pm(self, *args, **kw):
        got.setdefault("cf_plot", np.asarray(args[2], dtype=float).copy())  # first: ax[1]
        return orig_pm(self, *args, **kw)
    matplotlib.axes.Axes.pcolormesh = pm
    try:
        plot.dashboard(g.lam, spec.flux, np.zeros(len(g.lam)) * u.erg / u.cm ** 3 / u.s,
                       dtaus, g.pressures, T, th, g.opacities)
    finally:
        matplotlib.axes.Axes.pcolormesh = orig_pm
    out = dict(lam=g.lam.to(u.um).value, pressures=g.pressures.to(u.bar).value,
               spectrum=spec.flux.to(FLUX).value, final_T=T.to(u.K).value,
               dtaus=np.asarray(dtaus, dtype=float), p_milne=p_milne,
               T_milne=float(u.Quantity(t_milne).value),
               T_planck=float(t_planck.to(u.K).value), T_eff=float(t_eff.to(u.K).value),
               cf_plot=got["cf_plot"])
    dest = os.path.join(HERE, "post_c1.npz")
    np.savez_compressed(dest, **out)
    print(f"wrote post_c1.npz: {os.path.getsize(dest) / 1024:.1f} KiB; T_eff {out['T_eff']:.2f} K "
          f"(Milne {out['T_milne']:.2f}, Planck {out['T_planck']:.2f}), cf {got['cf_plot'].shape}")


if __name__ == "__main__":
    main()
