"""Import harness for the read-only reference (bmorris3/frei) — golden generation only.

Runs ONLY in the build container under ``/opt/conda/bin/python3.9`` (numpy 1.26,
astropy 4.3.1, scipy 1.7.1).  It never ships with the product and nothing on
the GPU box imports it.  It installs the stand-ins SURVEY.md Appendix B lists
(xarray, specutils, periodictable, expecto, numba-free ``frei.interp``) and a
stub parent package whose ``__path__`` points at ``/root/reference/frei`` so
the reference's own hot-path modules (``twostream``, ``opacity``, ``core``,
``tp``, ``chemistry``) load unmodified.

The xarray stand-in implements exactly what the hot path uses, following
xarray's published ``interp`` algorithm (sortby -> ``_localize`` +-2 nodes ->
``scipy.interpolate.interpn`` for >=2 dims / ``interp1d`` for 1 dim, ``fill_value``
honoured) and ``concat(...).sum()`` as a NaN-skipping numpy sum along the new
leading axis.  xarray itself is not installed anywhere in this image, so
``kappa``'s interpolation is pinned to this restatement of it
("Third-party arithmetic").
"""
import sys
import types
import warnings

warnings.filterwarnings("ignore")

import numpy as np  # noqa: E402

# --- 1. numpy aliases astropy 4.3.1 still uses --------------------------------
for _name, _val in dict(asscalar=lambda a: a.item(), alen=len, msort=np.sort,
                        float=float, int=int, bool=bool, object=object,
                        complex=complex, str=str).items():
    if not hasattr(np, _name):
        setattr(np, _name, _val)

import astropy.units as u  # noqa: E402
from astropy.units.quantity_helper import function_helpers as _fh  # noqa: E402


# --- 2. astropy's concatenate helper must accept numpy 1.26's dtype/casting ----
def _concatenate(arrays, axis=0, out=None, dtype=None, casting="same_kind"):
    arrays, kwargs, unit, out = _fh._iterable_helper(*arrays, out=out, axis=axis)
    return (arrays,), kwargs, unit, out


_fh.FUNCTION_HELPERS[np.concatenate] = _concatenate


# --- 3. xarray stand-in -------------------------------------------------------
class DataArray:
    __array_ufunc__ = None  # ndarray * DataArray -> DataArray.__rmul__

    def __init__(self, data, dims=None, coords=None, name=None):
        self.values = np.asarray(getattr(data, "value", data), dtype=float) \
            if not isinstance(data, DataArray) else data.values
        if isinstance(dims, str):
            dims = (dims,)
        self.dims = tuple(dims) if dims is not None else tuple(
            f"dim_{i}" for i in range(self.values.ndim))
        self.coords = {}
        for k, v in (coords or {}).items():
            self.coords[k] = np.asarray(getattr(v, "value", v), dtype=float)
        self.name = name

    def __getattr__(self, item):
        coords = self.__dict__.get("coords", {})
        if item in coords:
            return coords[item]
        raise AttributeError(item)

    @property
    def shape(self):
        return self.values.shape

    def _binop(self, other, op):
        o = other.values if isinstance(other, DataArray) else np.asarray(other)
        return DataArray(op(self.values, o), self.dims, self.coords)

    def __mul__(self, other):
        return self._binop(other, lambda a, b: a * b)

    def __rmul__(self, other):
        o = other.values if isinstance(other, DataArray) else np.asarray(other)
        return DataArray(o * self.values, self.dims, self.coords)

    def drop_duplicates(self, dim, keep="first"):
        ax = self.dims.index(dim)
        c = self.coords[dim]
        _, idx = np.unique(c, return_index=True)
        idx = np.sort(idx)
        coords = dict(self.coords)
        coords[dim] = c[idx]
        return DataArray(np.take(self.values, idx, axis=ax), self.dims, coords)

    def interp(self, coords=None, method="linear", assume_sorted=False,
               kwargs=None, **coords_kwargs):
        from scipy.interpolate import interpn, interp1d
        points = dict(coords or {})
        points.update(coords_kwargs)
        kwargs = dict(kwargs or {})
        fill_value = kwargs.get("fill_value", np.nan)
        idims = [d for d in self.dims if d in points]
        odims = [d for d in self.dims if d not in points]
        vals = np.transpose(self.values, [self.dims.index(d) for d in idims + odims])
        grids = []
        for k, d in enumerate(idims):
            # sortby (Dataset.interp, assume_sorted=False)
            x = self.coords[d]
            order = np.argsort(x, kind="stable")
            x = x[order]
            vals = np.take(vals, order, axis=k)
            # xarray.core.missing._localize: nearest index of min/max, +-2
            nx = np.asarray(points[d].values if isinstance(points[d], DataArray)
                            else points[d], dtype=float).ravel()
            imin = int(np.argmin(np.abs(x - np.nanmin(nx))))
            imax = int(np.argmin(np.abs(x - np.nanmax(nx))))
            sl = slice(max(imin - 2, 0), imax + 2)
            x = x[sl]
            vals = np.take(vals, np.arange(vals.shape[k])[sl], axis=k)
            grids.append(x)
        new = [np.asarray(points[d].values if isinstance(points[d], DataArray)
                          else points[d], dtype=float).ravel() for d in idims]
        if len(idims) == 1:
            f = interp1d(grids[0], vals, kind=method, axis=0, bounds_error=False,
                         fill_value=fill_value, assume_sorted=True)
            res = f(new[0])
        else:
            xi = np.stack(new, axis=-1)
            res = interpn(tuple(grids), vals, xi, method=method,
                          bounds_error=False, fill_value=fill_value)
        return DataArray(res, ("z",) + tuple(odims),
                         {d: self.coords[d] for d in odims if d in self.coords})

    def sum(self, dim):
        ax = self.dims.index(dim)
        v = np.where(np.isnan(self.values), 0.0, self.values)
        return DataArray(np.sum(v, axis=ax),
                         tuple(d for d in self.dims if d != dim), self.coords)


def concat(objs, dim):
    return DataArray(np.stack([o.values for o in objs], axis=0),
                     (dim,) + tuple(objs[0].dims), objs[0].coords)


_xr = types.ModuleType("xarray")
_xr.DataArray = DataArray
_xr.concat = concat
sys.modules["xarray"] = _xr

# --- 4. small third-party stand-ins -------------------------------------------
_pt = types.ModuleType("periodictable")


class _El:
    def __init__(self, mass):
        self.mass = mass


_pt.elements = types.SimpleNamespace(**{k: _El(v) for k, v in dict(
    H=1.00794, He=4.002602, C=12.0107, N=14.0067, O=15.9994, F=18.9984032,
    Na=22.98977, Al=26.981538, Cl=35.453, K=39.0983, Ti=47.867, V=50.9415,
    Cr=51.9961, Fe=55.845).items()})
sys.modules["periodictable"] = _pt


class Spectrum1D:
    def __init__(self, flux=None, spectral_axis=None):
        self.flux = flux
        self.spectral_axis = spectral_axis
        self.wavelength = spectral_axis


_su = types.ModuleType("specutils")
_su.Spectrum1D = Spectrum1D
sys.modules["specutils"] = _su
_ex = types.ModuleType("expecto")
_ex.get_spectrum = None
sys.modules["expecto"] = _ex

# --- 5. stub parent package + numba-free interp --------------------------------
REF = "/root/reference/frei"
_pkg = types.ModuleType("frei")
_pkg.__path__ = [REF]
sys.modules["frei"] = _pkg
_interp = types.ModuleType("frei.interp")
_interp.groupby_bins_agg = None
sys.modules["frei.interp"] = _interp

sys.dont_write_bytecode = True


def load():
    """Import and return the reference hot-path modules."""
    import importlib
    mods = {}
    for m in ("chemistry", "opacity", "twostream", "tp", "core"):
        mods[m] = importlib.import_module("frei." + m)
    return types.SimpleNamespace(**mods, u=u, DataArray=DataArray)
