"""A duck-typed stand-in for the reference's xarray.DataArray opacity tables (test
infrastructure; xarray is not importable here).  It carries what frei_amd reads from a table:
``.values``, the axis names ``.dims`` and the coordinates as attributes (``.pressure`` bar,
``.temperature`` K, ``.wavelength`` µm), like the DataArrays ``binned_opacity`` returns
(interp.py:287-307; opacity.py:137-146, 156-167)."""
import numpy as np


class DataArrayLike:
    def __init__(self, values, dims, **coords):
        self.values = np.asarray(values)
        self.dims = tuple(dims)
        assert self.values.ndim == len(self.dims)
        for name, c in coords.items():
            c = np.asarray(c, dtype=float)
            assert c.size == self.values.shape[self.dims.index(name)], name
            setattr(self, name, c)

    @property
    def shape(self):
        return self.values.shape


def reference_layouts(v_ptl, p, T, lam):
    """The three layouts the reference produces for one (pressure, temperature, wavelength)
    array: load_example_opacity's (p, T, λ), groupies' (T, p, λ), exact's (λ, T, p)."""
    co = dict(pressure=p, temperature=T, wavelength=lam)
    return {
        "ptl": DataArrayLike(v_ptl, ("pressure", "temperature", "wavelength"), **co),
        "tpl": DataArrayLike(np.transpose(v_ptl, (1, 0, 2)),
                             ("temperature", "pressure", "wavelength"), **co),
        "ltp": DataArrayLike(np.transpose(v_ptl, (2, 1, 0)),
                             ("wavelength", "temperature", "pressure"), **co),
    }
