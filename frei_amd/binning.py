"""Opacity binning on the GPU (frei/opacity.py:66-170 ``binned_opacity``; frei/interp.py
``groupby_bins_agg``; opacity.py:33-42 ``mapfunc_exact``).

A :class:`CrossSection` is one species' high-resolution cross-section in the layout the
reference's ``opacity_dir_to_netcdf`` writes (opacity.py:395-483): float32
``opacity[temperature][pressure][wavelength]`` with wavelengths in µm ascending.  It is
uploaded once per device and stays in HBM; K6 (``frei_amd/csrc/frei_binning.hip``) bins
it onto a Grid's wavelength bins and selects the nearest source (T, p) node for every
grid node.  ``binned_opacity`` returns :class:`BinnedTable` objects: the Engine bins them
straight into its device tables (no host round trip); ``.values`` materialises the
(pressure, temperature, wavelength) array on the host when asked.
"""
import ctypes
import glob
import os

import numpy as np

from . import _native as N
from .chemistry import iso_to_species
from .units import value

__all__ = ["CrossSection", "BinnedTable", "binned_opacity", "open_cross_section",
           "GROUPIES", "EXACT"]

GROUPIES, EXACT = 0, 1


class CrossSection:
    """High-resolution cross-section of one species (the reference's netCDF Dataset)."""

    def __init__(self, opacity, temperature, pressure, wavelength, isotopologue=None):
        self.opacity = np.ascontiguousarray(opacity, dtype=np.float32)
        self.temperature = np.ascontiguousarray(value(temperature, "K"), dtype=np.float64)
        self.pressure = np.ascontiguousarray(value(pressure, "bar"), dtype=np.float64)
        self.wavelength = np.ascontiguousarray(value(wavelength, "um"), dtype=np.float64)
        self.isotopologue = isotopologue
        self._synthetic = None
        if self.opacity.shape != (self.temperature.size, self.pressure.size,
                                  self.wavelength.size):
            raise ValueError("opacity must be (temperature, pressure, wavelength)")
        self._handles = {}

    @classmethod
    def synthetic(cls, temperature, pressure, wavelength, seed=0, isotopologue=None):
        """Device-generated line forest (benchmarks): no host copy of the values."""
        obj = cls.__new__(cls)
        obj.temperature = np.ascontiguousarray(temperature, dtype=np.float64)
        obj.pressure = np.ascontiguousarray(pressure, dtype=np.float64)
        obj.wavelength = np.ascontiguousarray(wavelength, dtype=np.float64)
        obj.opacity = None
        obj.isotopologue = isotopologue
        obj._synthetic = int(seed)
        obj._handles = {}
        return obj

    def handle(self, device=0):
        """frei_xsec* of this cross-section on ``device`` (uploaded once)."""
        h = self._handles.get(device)
        if h is None:
            lib = N.lib()
            h = ctypes.c_void_p()
            nT, npr, nhi = self.temperature.size, self.pressure.size, self.wavelength.size
            if self._synthetic is not None:
                N.check(lib.frei_xsec_create_synthetic(
                    ctypes.byref(h), device, nT, npr, nhi, N.dptr(self.temperature),
                    N.dptr(self.pressure), N.dptr(self.wavelength), self._synthetic))
            else:
                N.check(lib.frei_xsec_create(
                    ctypes.byref(h), device, N.fptr(self.opacity), nT, npr, nhi,
                    N.dptr(self.temperature), N.dptr(self.pressure), N.dptr(self.wavelength)))
            self._handles[device] = h
        return h

    def release(self):
        for h in self._handles.values():
            N.lib().frei_xsec_destroy(h)
        self._handles = {}

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass

    def bin(self, wl_bins, lam, temperatures, pressures, groupies=True, device=0, out=True):
        """Binned (pressure, temperature, λ) table on the host (``out=False``: leave it on
        the device, for timing)."""
        wl_bins = N.f64(value(wl_bins, "um"))
        lam = N.f64(value(lam, "um"))
        T = N.f64(value(temperatures, "K"))
        p = N.f64(value(pressures, "bar"))
        if wl_bins.size != lam.size + 1:
            raise ValueError("wl_bins must have one more edge than lam has points")
        res = np.empty((p.size, T.size, lam.size)) if out else None
        N.check(N.lib().frei_xsec_bin(self.handle(device), GROUPIES if groupies else EXACT,
                                      N.dptr(wl_bins), N.dptr(lam), lam.size, N.dptr(T), T.size,
                                      N.dptr(p), p.size, N.dptr(res)))
        return res

    def timing(self, on, device=0):
        ms, n = ctypes.c_double(0), ctypes.c_int(0)
        N.check(N.lib().frei_xsec_timing(self.handle(device), int(on), ctypes.byref(ms),
                                         ctypes.byref(n)))
        return ms.value, n.value


class BinnedTable:
    """A species' opacity binned onto a grid: nodes ``pressure`` (bar) x ``temperature``
    (K), wavelengths ``wavelength`` (µm).  The Engine bins it directly into HBM."""

    dims = ("pressure", "temperature", "wavelength")

    def __init__(self, xsec, wl_bins, lam, temperatures, pressures, groupies=True, device=0):
        self.xsec = xsec
        self.wl_bins = N.f64(value(wl_bins, "um"))
        self.wavelength = N.f64(value(lam, "um"))
        self.temperature = N.f64(value(temperatures, "K"))
        self.pressure = N.f64(value(pressures, "bar"))
        self.groupies = bool(groupies)
        self.device = device
        self._values = None

    @property
    def mode(self):
        return GROUPIES if self.groupies else EXACT

    @property
    def shape(self):
        return (self.pressure.size, self.temperature.size, self.wavelength.size)

    @property
    def values(self):
        if self._values is None:
            self._values = self.xsec.bin(self.wl_bins, self.wavelength, self.temperature,
                                         self.pressure, self.groupies, self.device)
        return self._values


def open_cross_section(path):
    """Read one species file: ``.npz`` (arrays opacity/temperature/pressure/wavelength) or a
    classic netCDF3 file with the opacity_dir_to_netcdf variables (scipy.io).  HDF5-based
    netCDF4 (the reference's zlib output) needs a reader this image lacks: convert it to
    .npz elsewhere."""
    iso = os.path.basename(path).split("_")[0]
    if path.endswith(".npz"):
        d = np.load(path, allow_pickle=False)
        return CrossSection(d["opacity"], d["temperature"], d["pressure"], d["wavelength"], iso)
    with open(path, "rb") as f:
        magic = f.read(4)
    if magic[:3] != b"CDF":
        raise ValueError(f"{path}: not a netCDF3 file (netCDF4/HDF5 cannot be read here; "
                         "convert to .npz with arrays opacity/temperature/pressure/wavelength)")
    from scipy.io import netcdf_file
    with netcdf_file(path, "r", mmap=False) as nc:
        v = nc.variables
        return CrossSection(np.array(v["opacity"][:]), np.array(v["temperature"][:]),
                            np.array(v["pressure"][:]), np.array(v["wavelength"][:]), iso)


def binned_opacity(temperatures, pressures, wl_bins, lam, groupies=True, species=None,
                   path=None, cross_sections=None, device=0):
    """Opacity for all available species binned to ``lam`` (opacity.py:66-170).

    ``cross_sections`` ({isotopologue: CrossSection}) replaces reading files from ``path``
    (default ``~/.frei/*.nc``, then ``*.npz``).  ``species`` filters by species name
    (``iso_to_species``, chemistry.py:13-21).  Returns {isotopologue: BinnedTable}."""
    if cross_sections is None:
        if path is None:
            path = os.path.join(os.path.expanduser("~"), ".frei", "*.nc")
        paths = sorted(glob.glob(path))
        if not paths and path.endswith(".nc"):
            paths = sorted(glob.glob(path[:-3] + ".npz"))
        cross_sections = {}
        for pth in paths:
            iso = os.path.basename(pth).split("_")[0]
            if species is None or iso_to_species(iso) in species:
                cross_sections[iso] = open_cross_section(pth)
    elif species is not None:
        cross_sections = {k: v for k, v in cross_sections.items()
                          if iso_to_species(k) in species}
    if not cross_sections:
        raise FileNotFoundError(f"no opacity cross-sections found at {path!r}")
    return {iso: BinnedTable(x, wl_bins, lam, temperatures, pressures, groupies, device)
            for iso, x in cross_sections.items()}
