"""Opacity tables, Rayleigh scattering and ``kappa`` (frei/opacity.py).

Tables are the reference's ``{isotopologue: DataArray(pressure, temperature, wavelength)}``
dict (opacity.py:272-342); here the value type is :class:`OpacityTable` (any object
with ``.values``, ``.pressure`` [bar], ``.temperature`` [K] works, e.g. an xarray
DataArray).  ``kappa`` evaluates on the GPU through the C ABI (frei_kappa).
"""
import numpy as np

from .constants import M_BAR_DEFAULT, UM
from .units import scalar, unit_of, value, with_unit

__all__ = ["OpacityTable", "SeparableTable", "kappa", "load_example_opacity",
           "rayleigh_H2", "rayleigh_He", "binned_opacity"]

N_REF_H2 = 2.68678e19   # cm^-3, opacity.py:23
N_REF_HE = 2.546899e19  # cm^-3, opacity.py:24


TABLE_DIMS = ("pressure", "temperature", "wavelength")


def table_values(tab):
    """A table's values as (pressure, temperature, wavelength).

    The reference's tables are xarray DataArrays whose axes are found by NAME — ``kappa``
    interpolates ``pressure=`` / ``temperature=`` (opacity.py:252-263) — and the three
    producers lay them out differently: ``load_example_opacity`` (pressure, temperature,
    wavelength) (opacity.py:338-342), ``binned_opacity(groupies=True)`` (temperature,
    pressure, wavelength) (interp.py:287-307, opacity.py:137-146) and the default
    ``binned_opacity(groupies=False)`` of ``Grid.load_opacities`` (wavelength, temperature,
    pressure) (opacity.py:42, 156-167).  A table carrying ``.dims`` is therefore transposed by
    name; one without ``.dims`` (a plain object with ``.values``) must already be (pressure,
    temperature, wavelength).  Dims other than those three names raise ValueError: on a Grid
    n_T = n_p, so a positional guess could silently swap p and T."""
    vals = np.asarray(tab.values)
    dims = getattr(tab, "dims", None)
    if dims is None:
        return vals
    dims = tuple(str(d) for d in dims)
    if len(dims) != vals.ndim or sorted(dims) != sorted(TABLE_DIMS):
        raise ValueError(f"opacity table dims {dims} are not a permutation of {TABLE_DIMS}")
    return np.transpose(vals, [dims.index(d) for d in TABLE_DIMS])


class OpacityTable:
    """(pressure, temperature, wavelength) opacity grid in cm^2 g^-1.

    ``dims`` names the axes of ``values`` when they come in another order (e.g. a reference
    DataArray's ``.dims``); the values are stored transposed to (pressure, temperature,
    wavelength).  :meth:`from_dataarray` takes any object with ``.values``, ``.dims``,
    ``.pressure`` (bar), ``.temperature`` (K) and optionally ``.wavelength`` (µm)."""

    dims = TABLE_DIMS

    @classmethod
    def from_dataarray(cls, da):
        wl = getattr(da, "wavelength", None)
        return cls(table_values(da), np.asarray(da.pressure), np.asarray(da.temperature),
                   None if wl is None else np.asarray(wl))

    def __init__(self, values, pressure, temperature, wavelength=None, dims=None):
        values = np.asarray(values, dtype=np.float64)
        if dims is not None:
            values = table_values(_Dimmed(values, dims))
        self.values = values
        self.pressure = np.asarray(value(pressure, "bar"), dtype=np.float64)
        self.temperature = np.asarray(value(temperature, "K"), dtype=np.float64)
        self.wavelength = None if wavelength is None else np.asarray(value(wavelength, "um"))
        if self.values.shape[:2] != (self.pressure.size, self.temperature.size):
            raise ValueError("values must be (n_pressure, n_temperature, n_wavelength)")

    @property
    def shape(self):
        return self.values.shape

    def drop_duplicates(self, dim="temperature"):
        """Keep the first of repeated temperature nodes (xarray drop_duplicates)."""
        if dim != "temperature":
            raise ValueError("only temperature duplicates are dropped")
        _, idx = np.unique(self.temperature, return_index=True)
        idx = np.sort(idx)
        return OpacityTable(self.values[:, idx], self.pressure, self.temperature[idx],
                            self.wavelength)


class _Dimmed:
    def __init__(self, values, dims):
        self.values, self.dims = values, dims


class SeparableTable:
    """Synthetic table generated on the device: clip((fp[p] * fT[T]) * base[lam], lo, hi).
    Used for large benchmark grids (no host copy of the n_p*n_T*n_lam values)."""

    def __init__(self, base, fp, fT, pressure, temperature, lo=1e-4, hi=1e3):
        self.base = np.ascontiguousarray(base, dtype=np.float64)
        self.fp = np.ascontiguousarray(fp, dtype=np.float64)
        self.fT = np.ascontiguousarray(fT, dtype=np.float64)
        self.pressure = np.asarray(value(pressure, "bar"), dtype=np.float64)
        self.temperature = np.asarray(value(temperature, "K"), dtype=np.float64)
        self.lo, self.hi = float(lo), float(hi)

    @property
    def values(self):  # materialise on the host (small grids / tests only)
        return np.clip((self.fp[:, None] * self.fT[None, :])[:, :, None] * self.base[None, None, :],
                       self.lo, self.hi)


def n_lambda_H2(lam_um):
    """Malik 2017 Eqn 17 (opacity.py:173-177); lam in µm."""
    return 13.58e-5 * (1 + (7.52e-11 * np.asarray(lam_um) ** -2) * 1e8) + 1


def n_lambda_He(lam_um):
    """Deitrick 2020 Eqn C3 (opacity.py:180-184); lam in µm."""
    return 1e-8 * (2283 + (1.8102e13 / (1.5342e10 - np.asarray(lam_um) ** -2))) + 1


def _rayleigh(n, n_ref, lam_cm, m_bar):
    return (24 * np.pi ** 3 / n_ref ** 2 / lam_cm ** 4 *
            ((n ** 2 - 1) / (n ** 2 + 2)) ** 2 * 1) / m_bar


def rayleigh_H2(wavelength, m_bar=M_BAR_DEFAULT):
    """Rayleigh cross-section per unit mass, cm^2 g^-1 (opacity.py:187-192); lam in µm."""
    lam = value(wavelength, "um")
    return _rayleigh(n_lambda_H2(lam), N_REF_H2, lam * UM, scalar(m_bar, "g"))


def rayleigh_He(wavelength, m_bar=M_BAR_DEFAULT):
    """(opacity.py:195-200)"""
    lam = value(wavelength, "um")
    return _rayleigh(n_lambda_He(lam), N_REF_HE, lam * UM, scalar(m_bar, "g"))


def sigma_scattering(lam_um, m_bar):
    """rayleigh_H2 + rayleigh_He (opacity.py:233)."""
    return rayleigh_H2(lam_um, m_bar) + rayleigh_He(lam_um, m_bar)


_KAPPA_P = np.array([4.0, 2.0, 1.0, 0.5])   # bar: kappa's context needs some layer grid


def kappa(opacities, temperature, pressure, lam, m_bar=M_BAR_DEFAULT, device=0,
          chemistry=None):
    """Total opacity at one (T, p): (k, sigma_scattering) in cm^2 g^-1 (opacity.py:203-269).

    k = sum_s mmr_s * interp_s(p, T) + sigma (linear, fill 0 outside the node hull;
    pressure-only for single-temperature tables).  mmr_s = ``chemistry(T, p, species,
    m_bar=m_bar)`` at the query point (opacity.py:246-248) when a provider is given, else the
    reference's mock.  Runs on the GPU."""
    from .chemistry import provider_mmr
    from .engine import cached_engine
    lam_um = np.asarray(value(lam, "um"), dtype=float)
    T = np.asarray(value(temperature, "K"), dtype=float)
    p = np.asarray(value(pressure, "bar"), dtype=float)
    mb = scalar(m_bar, "g")
    # one context per (tables, wavelengths, m_bar), reused across calls; its layer grid only
    # carries the mixing ratios: the mock's (layer-independent), or the provider's at each
    # query point, set before the query
    eng = cached_engine(opacities, lam_um=lam_um, p_bar=_KAPPA_P, g=1.0, m_bar=mb, F_toa=None,
                        device=device, tag=None if chemistry is None else ("kappa", id(chemistry)))
    names = list(opacities)

    # Quantities in -> (k, sigma) in cm^2 g^-1 Quantities out (opacity.py:269)
    ku = unit_of("cm2 / g", temperature, pressure, lam, m_bar)

    def query(Tq, pq):
        if chemistry is not None:
            m = provider_mmr(chemistry, [Tq], [pq], names, mb)[:, 0]
            eng.set_mmr(np.repeat(m[:, None], _KAPPA_P.size, axis=1))
        return eng.kappa(Tq, pq)
    if T.ndim == 0 and p.ndim == 0:
        k, sig = query(float(T), float(p))
        return with_unit(k, ku), with_unit(sig, ku)
    # vector mode: points along one dimension z (opacity.py:235-263).  The reference
    # flattens the (z, lam) result before adding sigma (opacity.py:266-269), so a one-point
    # array gives a flat k; for z > 1 its broadcast fails, and here k is (z, lam).
    Tz, pz = np.broadcast_arrays(T, p)
    ks = []
    sig = None
    for Tq, pq in zip(Tz.ravel(), pz.ravel()):
        k, sig = query(float(Tq), float(pq))
        ks.append(k)
    k = ks[0] if len(ks) == 1 else np.array(ks).reshape(Tz.shape + (lam_um.size,))
    return with_unit(k, ku), with_unit(sig, ku)


def load_example_opacity(grid, seed=42, scale_factor=20):
    """Synthetic "example" water opacity (opacity.py:272-342): broad IR/optical bands,
    15 random optical lines (np.random.seed(seed)) and 3 NIR bands, identical at every
    (p, T) node of ``grid``."""
    lam = np.asarray(grid.lam, dtype=float)
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
    row *= scale_factor
    p = np.asarray(grid.pressures, dtype=float)
    T = np.asarray(grid.init_temperatures, dtype=float)
    vals = np.broadcast_to(row, (p.size, T.size, lam.size))
    return {"1H2-16O": OpacityTable(vals, p, T, lam).drop_duplicates("temperature")}


def binned_opacity(temperatures, pressures, wl_bins, lam, groupies=True, species=None,
                   path=None, **kwargs):
    """Bin high-resolution cross-sections onto ``lam`` (opacity.py:66-170) on the GPU;
    see :func:`frei_amd.binning.binned_opacity`."""
    from .binning import binned_opacity as _bo
    return _bo(temperatures, pressures, wl_bins, lam, groupies=groupies, species=species,
               path=path, **kwargs)
