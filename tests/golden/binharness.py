"""Import harness for the reference's opacity-binning path — golden generation only.

Runs ONLY in the build container under ``/opt/conda/bin/python3.9`` after
``refharness`` (which installs the hot-path stand-ins of SURVEY.md Appendix B).  It
lets the reference's own ``frei/opacity.py::binned_opacity`` (both the default
``groupies=True`` branch and the ``groupies=False`` / ``mapfunc_exact`` branch of
``Grid.load_opacities``) and its own ``frei/interp.py`` (``groupby_bins_agg``,
``AggregateTrapz``) run unmodified, by standing in for the third-party packages the
image lacks:

* ``numba`` — ``njit`` is the identity, so interp.py's trapezoid loop runs as plain
  Python on numpy float32 scalars.  numba would promote ``(a + b) / 2`` to float64 and
  round the float32 accumulator once per addition; both round to the same float32
  unless the exact sum needs more than 53 bits (accumulator/term exponent gap > 29),
  which no fixture reaches (the goldens test checks the oracle's numba semantics
  bit-for-bit against this run).
* ``numpy_groupies`` (unpinned) — the pieces interp.py imports, restated from the
  package's published algorithm: ``input_validation`` (axis=-1 "offset" labels, C-order
  ravel), ``check_dtype`` (unknown functions such as 'trapz' keep the input dtype, so
  the accumulator is float32), ``get_func``/``get_aliasing``.
* ``xarray`` — the DataArray/Dataset operations the binning path calls, following
  xarray's published semantics: ``where(drop=True)``, ``apply_ufunc`` (core dims moved
  last), ``groupby_bins(...).map`` (pandas.cut, right-closed bins, empty bins dropped,
  results concatenated in bin order), ``interp`` (sortby, ``_localize``, decomposed
  into orthogonal 1-D scipy ``interp1d`` calls), ``integrate`` (duck_array_ops.trapz:
  ``dx * 0.5 * (y[1:] + y[:-1])`` summed), ``expand_dims``.
* ``pandas`` is the real one (conda python3.9), so bin assignment is pinned to
  ``pd.cut`` itself.

Nothing here ships with the product; the GPU box never imports it.
"""
import glob
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refharness  # noqa: E402,F401  (base stand-ins, stub parent package)

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402


# --- numba: identity jit ----------------------------------------------------------
def _njit(f=None, **kw):
    return f if f is not None else (lambda g: g)


_nb = types.ModuleType("numba")
_nb.njit = _njit
sys.modules["numba"] = _nb

# --- numpy_groupies stand-ins ---------------------------------------------------------
_ng = types.ModuleType("numpy_groupies")
_ng_utils = types.ModuleType("numpy_groupies.utils")
_ng_utils.funcs_common = ["first", "last", "len", "mean", "var", "std", "allnan", "anynan",
                          "max", "min", "argmax", "argmin", "sumofsquares", "cumsum",
                          "cumprod", "cummax", "cummin"]
_ng_np = types.ModuleType("numpy_groupies.utils_numpy")
_ng_np._alias_numpy = {np.add: "sum", np.sum: "sum", np.prod: "prod", np.mean: "mean",
                       np.max: "max", np.min: "min"}
_ng_agg = types.ModuleType("numpy_groupies.aggregate_numba")


def _get_aliasing(*extra):
    alias = {k: k for k in _ng_utils.funcs_common + ["sum", "prod", "all", "any"]}
    for e in extra:
        alias.update(e)
    return alias


def _input_validation(group_idx, a, size=None, order="C", axis=None, ravel_group_idx=True,
                      check_bounds=True, func=None):
    a = np.asanyarray(a)
    group_idx = np.asanyarray(group_idx)
    if not np.issubdtype(group_idx.dtype, np.integer):
        raise TypeError("group_idx must be of integer type")
    if check_bounds and np.any(group_idx < 0):
        raise ValueError("negative indices not supported")
    ndim_a = np.ndim(a)
    if axis is None:
        if ndim_a > 1:
            raise ValueError("a must be scalar or 1 dimensional")
        size = int(np.max(group_idx)) + 1 if size is None else size
        return group_idx, a, size, 1, size, None
    axis = axis if axis >= 0 else ndim_a + axis
    if a.shape[axis] != len(group_idx):
        raise ValueError("a.shape[axis] doesn't match length of group_idx.")
    size_in = int(np.max(group_idx)) + 1 if size is None else size
    shape = list(a.shape)
    shape[axis] = size_in
    # broadcast labels over the other axes and ravel in C order ("offset" method)
    idx = [np.arange(s).reshape([-1 if i == ii else 1 for i in range(ndim_a)])
           if ii != axis else group_idx.reshape([-1 if i == ii else 1 for i in range(ndim_a)])
           for ii, s in enumerate(a.shape)]
    idx = np.broadcast_arrays(*idx)
    flat = np.ravel_multi_index(idx, shape, order=order)
    return flat.ravel(), a.ravel(), int(np.prod(shape)), ndim_a, tuple(shape), None


def _check_dtype(dtype, func_str, a, n):
    if dtype is not None:
        return np.dtype(dtype)
    forced = {"len": np.int64, "nanlen": np.int64, "all": bool, "any": bool,
              "allnan": bool, "anynan": bool, "argmax": np.int64, "argmin": np.int64}
    if func_str in forced:
        return np.dtype(forced[func_str])
    if func_str in ("mean", "var", "std", "nanmean", "nanvar", "nanstd"):
        return a.dtype if np.issubdtype(a.dtype, np.floating) else np.dtype(np.float64)
    return a.dtype


def _check_fill_value(fill_value, dtype, func=None):
    np.dtype(dtype).type(fill_value)


def _get_func(func, aliasing, implementations):
    try:
        func_str = aliasing[func]
    except (KeyError, TypeError):
        if callable(func):
            return func
        raise ValueError(f"func {func} is neither a valid function string nor callable")
    if func_str in implementations:
        return func_str
    raise NotImplementedError("No such function available")


class _NGOp:
    def __init__(self, func=None, **kw):
        self.func = func


for _n in ("Sum", "Prod", "Len", "All", "Any", "Last", "First", "AllNan", "AnyNan", "Min",
           "Max", "ArgMin", "ArgMax", "Mean", "Std", "Var", "CumSum", "CumProd", "CumMax",
           "CumMin"):
    setattr(_ng_agg, _n, type(_n, (_NGOp,), {}))
_ng_agg.funcs_no_separate_nan = frozenset(["argmax", "argmin", "all", "any", "first", "last",
                                           "len", "cumsum", "cumprod", "cummax", "cummin"])
_ng_agg.check_dtype = _check_dtype
_ng_agg.check_fill_value = _check_fill_value
_ng_agg.get_func = _get_func
_ng_agg.isstr = lambda s: isinstance(s, str)
_ng_agg._default_cache = {}
_ng_np.input_validation = _input_validation
_ng_np.get_aliasing = _get_aliasing
_ng.utils = _ng_utils
_ng.utils_numpy = _ng_np
_ng.aggregate_numba = _ng_agg
for _m, _o in (("numpy_groupies", _ng), ("numpy_groupies.utils", _ng_utils),
               ("numpy_groupies.utils_numpy", _ng_np),
               ("numpy_groupies.aggregate_numba", _ng_agg)):
    sys.modules[_m] = _o


# --- xarray: dtype-preserving DataArray/Dataset for the binning path ----------------
def _vals(o):
    return o.values if isinstance(o, XArr) else np.asarray(o)


class XArr:
    """DataArray stand-in that keeps the dtype (float32 cross-sections stay float32)."""
    __array_ufunc__ = None

    def __init__(self, data, dims, coords=None, name=None):
        self.values = np.asarray(data)
        self.dims = tuple(dims)
        self.coords = dict(coords or {})
        self.name = name

    def __getattr__(self, item):
        coords = self.__dict__.get("coords", {})
        if item in coords:
            c = coords[item]
            d = (item,) if np.ndim(c) == 1 else ()
            return XArr(c, d, {item: c} if d else {}, name=item)
        raise AttributeError(item)

    def __array__(self, dtype=None):
        return self.values if dtype is None else self.values.astype(dtype)

    @property
    def shape(self):
        return self.values.shape

    @property
    def dtype(self):
        return self.values.dtype

    def _like(self, data):
        return XArr(data, self.dims, self.coords, self.name)

    def _bin(self, o, op, rev=False):
        if isinstance(o, XArr) and o.dims and o.dims != self.dims:
            raise NotImplementedError("broadcast by name not needed on this path")
        a, b = self.values, _vals(o)
        return self._like(op(b, a) if rev else op(a, b))

    def __gt__(self, o): return self._bin(o, np.greater)
    def __lt__(self, o): return self._bin(o, np.less)
    def __and__(self, o): return self._bin(o, np.logical_and)
    def __mul__(self, o): return self._bin(o, lambda a, b: a * b)
    def __rmul__(self, o): return self._bin(o, lambda a, b: a * b, rev=True)
    def __sub__(self, o): return self._bin(o, lambda a, b: a - b)
    def __truediv__(self, o): return self._bin(o, lambda a, b: a / b)

    def max(self): return XArr(np.max(self.values), ())
    def min(self): return XArr(np.min(self.values), ())
    def mean(self): return XArr(np.mean(self.values), ())

    def copy(self, data=None):
        return XArr(self.values.copy() if data is None else data, self.dims, self.coords,
                    self.name)

    def isel(self, dim, idx):
        ax = self.dims.index(dim)
        coords = {k: (v[idx] if k == dim else v) for k, v in self.coords.items()}
        return XArr(np.take(self.values, idx, axis=ax), self.dims, coords, self.name)

    def where(self, cond, drop=False):
        c = _vals(cond)
        if not drop:
            raise NotImplementedError
        (dim,) = cond.dims
        keep = np.nonzero(c)[0]
        out = self.isel(dim, keep)
        # where() itself: NaN where cond is False (none left after the drop)
        m = np.take(c, keep)
        shape = [1] * out.values.ndim
        shape[out.dims.index(dim)] = -1
        v = np.where(m.reshape(shape), out.values, np.nan).astype(out.values.dtype)
        return out._like(v)

    def rename(self, mapping):
        dims = tuple(mapping.get(d, d) for d in self.dims)
        coords = {mapping.get(k, k): v for k, v in self.coords.items()}
        return XArr(self.values, dims, coords, self.name)

    def interp(self, coords=None, method="linear", assume_sorted=False, kwargs=None,
               **coords_kwargs):
        return _interp(self, dict(coords or {}, **coords_kwargs), method, kwargs or {})

    def integrate(self, dim):
        # duck_array_ops.trapz: integrand = dx * 0.5 * (y[1:] + y[:-1]), summed (skipna=False)
        ax = self.dims.index(dim)
        x = self.coords[dim]
        y = np.moveaxis(self.values, ax, -1)
        dx = x[1:] - x[:-1]
        integrand = dx * 0.5 * (y[..., 1:] + y[..., :-1])
        val = np.sum(integrand, axis=-1)
        dims = tuple(d for d in self.dims if d != dim)
        return XArr(val, dims, {k: v for k, v in self.coords.items() if k != dim})

    def expand_dims(self, mapping):
        (dim, vals), = mapping.items()
        c = np.array([float(_vals(v)) for v in vals])
        coords = dict(self.coords)
        coords[dim] = c
        return XArr(self.values[None], (dim,) + self.dims, coords, self.name)


def _interp1d_dim(arr, dim, new, method, kwargs):
    from scipy.interpolate import interp1d
    ax = arr.dims.index(dim)
    x = np.asarray(arr.coords[dim], dtype=float)
    y = arr.values
    order = np.argsort(x, kind="stable")          # sortby
    x, y = x[order], np.take(y, order, axis=ax)
    if method in ("linear", "nearest") and x.size > 1:  # missing._localize
        imin = int(pd.Index(x).get_indexer([np.nanmin(new)], method="nearest")[0])
        imax = int(pd.Index(x).get_indexer([np.nanmax(new)], method="nearest")[0])
        sl = slice(max(imin - 2, 0), imax + 2)
        x, y = x[sl], np.take(y, np.arange(y.shape[ax])[sl], axis=ax)
    f = interp1d(x, y, kind=method, axis=ax, bounds_error=False,
                 fill_value=kwargs.get("fill_value", np.nan), assume_sorted=True, copy=False)
    coords = dict(arr.coords)
    coords[dim] = new
    return XArr(f(new), arr.dims, coords, arr.name)


def _interp(arr, points, method, kwargs):
    # orthogonal 1-D targets: xarray decomposes into independent 1-D interpolations
    out = arr
    for dim in [d for d in arr.dims if d in points]:
        out = _interp1d_dim(out, dim, np.asarray(_vals(points[dim]), dtype=float).ravel(),
                            method, kwargs)
    return out


class XDataset:
    def __init__(self, data_vars, coords):
        self.data_vars = data_vars
        self.coords = coords

    def __getattr__(self, item):
        dv = self.__dict__.get("data_vars", {})
        if item in dv:
            return dv[item]
        co = self.__dict__.get("coords", {})
        if item in co:
            return XArr(co[item], (item,), {item: co[item]}, name=item)
        raise AttributeError(item)

    def isel(self, dim, idx):
        coords = {k: (v[idx] if k == dim else v) for k, v in self.coords.items()}
        return XDataset({k: v.isel(dim, idx) for k, v in self.data_vars.items()}, coords)

    def interp(self, coords=None, method="linear", kwargs=None, **kw):
        dv = {k: v.interp(coords, method=method, kwargs=kwargs, **kw)
              for k, v in self.data_vars.items()}
        first = next(iter(dv.values()))
        return XDataset(dv, dict(first.coords))

    def groupby_bins(self, dim, bins):
        return _GroupByBins(self, dim, bins)


class _GroupByBins:
    def __init__(self, ds, dim, bins):
        self.ds, self.dim = ds, dim
        codes = pd.cut(np.asarray(ds.coords[dim]), bins).codes
        self.groups = [np.nonzero(codes == c)[0] for c in np.unique(codes[codes >= 0])]

    def map(self, func, **kwargs):
        parts = [func(self.ds.isel(self.dim, idx), **kwargs) for idx in self.groups]
        return _concat(parts, self.dim)


def _concat(objs, dim):
    ax = objs[0].dims.index(dim)
    coords = dict(objs[0].coords)
    coords[dim] = np.concatenate([o.coords[dim] for o in objs])
    return XArr(np.concatenate([o.values for o in objs], axis=ax), objs[0].dims, coords)


def apply_ufunc(func, *args, input_core_dims=None, output_core_dims=None, kwargs=None,
                **_):
    datas = []
    for a, core in zip(args, input_core_dims):
        other = [d for d in a.dims if d not in core]
        datas.append(np.transpose(a.values, [a.dims.index(d) for d in other + list(core)]))
    first = args[0]
    other = [d for d in first.dims if d not in input_core_dims[0]]
    res = func(*datas, **(kwargs or {}))
    coords = {k: v for k, v in first.coords.items() if k in other}
    return XArr(res, tuple(other) + tuple(output_core_dims[0]), coords)


_REGISTRY = {}


def open_dataset(path, **kw):
    return _REGISTRY[os.path.abspath(path)]


_xr = sys.modules["xarray"]
_xr.apply_ufunc = apply_ufunc
_xr.open_dataset = open_dataset

# --- real frei.interp (numba/numpy_groupies now stand in) ------------------------------
sys.modules.pop("frei.interp", None)


def register(directory, isotopologue, opacity, temperature, pressure, wavelength):
    """Create ``<directory>/<iso>_golden.nc`` (empty placeholder for glob) whose
    open_dataset is the opacity_dir_to_netcdf layout (opacity.py:466-479)."""
    os.makedirs(directory, exist_ok=True)
    path = os.path.abspath(os.path.join(directory, f"{isotopologue}_golden.nc"))
    open(path, "w").close()
    _REGISTRY[path] = XDataset(
        {"opacity": XArr(opacity, ("temperature", "pressure", "wavelength"),
                         dict(temperature=temperature, pressure=pressure,
                              wavelength=wavelength), name="opacity")},
        dict(temperature=temperature, pressure=pressure, wavelength=wavelength))
    return path


def load():
    import importlib
    R = refharness.load()
    R.interp = importlib.import_module("frei.interp")
    return R


__all__ = ["load", "register", "glob"]
