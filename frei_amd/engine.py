"""Host driver of one GPU context (one ``frei_ctx`` of include/frei_hip.h).

An :class:`Engine` owns a contiguous wavelength slice of a global grid on one device:
it precomputes the per-wavelength constants of the reference's setup (Planck prefactor,
Rayleigh sigma, F_TOA, trapezoid weights — core.py:48-62, opacity.py:173-200,
twostream.py:16-20, 46-67) with NumPy on the host, uploads the opacity tables and mmr,
and calls the HIP kernels for sweeps, the T-P loop and kappa.  Nothing here computes
fluxes on the CPU: without libfrei_hip.so every call raises.
"""
import ctypes
import os

import numpy as np

from . import _native as N
from .binning import BinnedTable
from .chemistry import ChemistryTable, fixed_provider_mmr, provider_mmr
from .chemistry import chemistry as mock_chemistry
from .constants import BAR, C, H, K_B, M_BAR_DEFAULT, UM
from .opacity import SeparableTable, sigma_scattering, table_values
from .units import scalar, value

EMIT, ABSORB = 0, 1


def planck_prefactor(lam_cm):
    """2 h c^2 / lam^5 exactly as BB forms it (twostream.py:64-66)."""
    return 2 * H * C ** 2 / np.power(lam_cm, 5)


def bb(T, lam_um):
    lam_cm = np.asarray(lam_um, dtype=float) * UM
    return planck_prefactor(lam_cm) / np.expm1(H * C / (lam_cm * K_B * T))


def f_toa(lam_um, T_star=5800.0, f=2 / 3, a_rstar=6.450964670116429):
    """Stellar flux at the top of the atmosphere, erg s^-1 cm^-3 (core.py:48-55)."""
    return f * a_rstar ** -2 * 1 / (2 * np.pi) * (np.pi * bb(T_star, lam_um))


def trapz_weights(lam_cm):
    """Per-point trapezoid weights of np.trapz on the global grid, so a wavelength slice
    contributes sum(w*F) with no halo."""
    d = np.diff(lam_cm)
    w = np.zeros(lam_cm.size)
    w[:-1] += d / 2
    w[1:] += d / 2
    return w


def partition(n, nranks, rank):
    """Contiguous, balanced wavelength slice [lo, hi) of rank ``rank``."""
    base, rem = divmod(n, nranks)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def balanced_edges(edges, costs, align=256):
    """Slice edges of equal measured cost.

    ``edges`` = [0, e_1, ..., n]: the current contiguous slices, ``costs`` = each slice's
    measured time (e.g. its sweep kernel's).  The cost per wavelength is taken as constant inside
    each current slice, and the new edges split the cumulative cost into equal parts, rounded to
    multiples of ``align`` wavelengths (whole sweep blocks) and kept strictly increasing.  The
    per-wavelength work of the sweep depends on the data (the opacities, the temperatures), so
    an even split leaves some ranks on the critical path of every exchange.
    """
    edges = np.asarray(edges, dtype=np.int64)
    costs = np.asarray(costs, dtype=float)
    R, n = len(costs), int(edges[-1])
    if len(edges) != R + 1 or np.any(np.diff(edges) <= 0) or np.any(costs <= 0):
        raise ValueError("edges must increase and bound len(costs) slices of positive cost")
    cum = np.concatenate([[0.0], np.cumsum(costs)])          # cumulative cost at the edges
    out = [0]
    for k in range(1, R):
        x = float(np.interp(cum[-1] * k / R, cum, edges))   # piecewise-linear inverse
        e = int(round(x / align)) * align
        e = min(max(e, out[-1] + align), n - (R - k) * align)
        out.append(e)
    out.append(n)
    return out


def _table_arrays(tab):
    p = np.asarray(value(tab.pressure, "bar"), dtype=float)
    T = np.asarray(value(tab.temperature, "K"), dtype=float)
    return p, T


def device_key(device):
    """Host name and PCI bus id of ``device``: equal for ranks that share one GPU."""
    import socket
    buf = ctypes.create_string_buffer(64)
    N.check(N.lib().frei_device_pci_bus_id(int(device), buf, 64))
    return f"{socket.gethostname()}|{buf.value.decode()}"


class Engine:
    """One device context for the wavelength slice ``lam_slice`` of ``lam_um``.

    Parameters mirror the reference's Grid/Planet: ``p_bar`` layer pressures (bar,
    descending), ``opacities`` dict of tables, ``g`` (cm s^-2), ``m_bar`` (g),
    ``F_toa`` (erg s^-1 cm^-3, global grid) and ``mmr`` [n_species][n_layers]
    (default: the reference's mock chemistry, chemistry.py:207-246) or a
    :class:`~frei_amd.chemistry.ChemistryTable` (T-dependent, re-evaluated every sweep), or
    ``chemistry``: a provider on the reference's signature ``chemistry(T, p, species,
    m_bar=...)`` (frei_amd.chemistry, "chemistry providers"), evaluated where the reference's
    kappa evaluates it.
    """

    def __init__(self, lam_um, p_bar, opacities, g=2478.6519476149147, m_bar=M_BAR_DEFAULT,
                 F_toa=None, mmr=None, device=0, lam_slice=None, comm=None, chemistry=None):
        lib = N.lib()
        self.lam_um = np.asarray(value(lam_um, "um"), dtype=float)
        self.p_bar = np.asarray(value(p_bar, "bar"), dtype=float)
        self.g = scalar(g, "cm / s2")
        self.m_bar = scalar(m_bar, "g")
        self.names = list(opacities)
        self.n_layers = self.p_bar.size
        n = self.lam_um.size
        lo, hi = lam_slice if lam_slice is not None else (0, n)
        self.lo, self.hi = lo, hi
        self.n_lam = hi - lo
        self.device = device
        lam_cm = self.lam_um * UM
        sl = slice(lo, hi)
        self.c1 = N.f64(planck_prefactor(lam_cm)[sl])
        self.lk = N.f64((lam_cm * K_B)[sl])
        self.sigma = N.f64(sigma_scattering(self.lam_um, self.m_bar)[sl])
        ft = f_toa(self.lam_um) if F_toa is None else value(F_toa, "erg / (s cm3)")
        self.f_toa = N.f64(np.asarray(ft, dtype=float)[sl])
        self.wtr = N.f64(trapz_weights(lam_cm)[sl])
        self.p_cgs = N.f64(self.p_bar * BAR)
        ctx = ctypes.c_void_p()
        N.check(lib.frei_ctx_create(ctypes.byref(ctx), device, self.n_layers, self.n_lam,
                                    len(self.names)))
        self._ctx = ctx
        N.check(lib.frei_set_grid(ctx, N.dptr(self.c1), N.dptr(self.lk), N.dptr(self.sigma),
                                  N.dptr(self.f_toa), N.dptr(self.wtr), N.dptr(self.p_cgs),
                                  self.g, self.m_bar))
        for s, name in enumerate(self.names):
            self._set_table(s, opacities[name], sl)
        # a chemistry provider (the reference's chemistry(T, p, species, m_bar)): fixed per-layer
        # mixing ratios when it does not depend on T, else evaluated between sweeps (run)
        self.provider = None
        provider = chemistry
        if provider is not None:
            if mmr is not None:
                raise ValueError("pass either mmr or a chemistry provider, not both")
            mmr = fixed_provider_mmr(provider, self.names, self.p_bar, self.m_bar)
            if mmr is None:
                self.provider = provider
                mmr = provider_mmr(provider, np.full(self.n_layers, 1000.0), self.p_bar,
                                   self.names, self.m_bar)
        chem = mmr if isinstance(mmr, ChemistryTable) else None
        if mmr is None or chem is not None:
            T0 = np.full(self.n_layers, 1000.0)
            mm = mock_chemistry(T0, self.p_bar, self.names, m_bar=self.m_bar)
            mmr = np.array([mm[nm] for nm in self.names])
        self.mmr = N.f64(np.broadcast_to(np.asarray(mmr, dtype=float),
                                         (len(self.names), self.n_layers)))
        N.check(lib.frei_set_mmr(ctx, N.dptr(self.mmr)))
        self.chemistry = chem
        if chem is not None:   # T-dependent chemistry, re-evaluated on the device every sweep
            v = N.f64(chem.array(self.names))
            N.check(lib.frei_set_chemistry(ctx, N.dptr(v), N.dptr(N.f64(chem.temperature)),
                                           chem.temperature.size,
                                           N.dptr(N.f64(chem.pressure * BAR)),
                                           chem.pressure.size))
        if self.provider is not None:
            # mixing ratios change every sweep: the per-species sum in the sweep (the reference's
            # own order) instead of a species contraction rebuilt per sweep
            self.set_option("precontract", 0)
        self._ag_keep = None
        if comm is not None:
            self._join(comm)

    def _join(self, comm):
        """comm = ("rccl", nranks, rank, unique_id_bytes),
        ("p2p", nranks, rank, all_gather(bytes) -> [bytes] in rank order) or
        ("host", nranks, rank, allgather(send: ndarray) -> ndarray[nranks * n])."""
        lib = N.lib()
        kind, nranks, rank, arg = comm
        if kind == "rccl":
            buf = ctypes.create_string_buffer(bytes(arg), 128)
            N.check(lib.frei_comm_init(self._ctx, nranks, rank, buf))
        elif kind == "p2p":
            h = ctypes.create_string_buffer(64)
            # FREI_FAULT_P2P=1: fault injection for the fallback tests (this rank's setup fails,
            # it still joins the handle exchange so its peers fail too instead of hanging)
            if os.environ.get("FREI_FAULT_P2P") == "1":
                rc, msg = 1, "P2P setup failure injected (FREI_FAULT_P2P)"
            else:
                rc = lib.frei_comm_p2p_handle(self._ctx, nranks, rank, h)
                msg = lib.frei_last_error().decode(errors="replace") if rc else ""
            hs = arg(h.raw if rc == 0 else b"")     # every rank joins the exchange
            if rc != 0:
                raise RuntimeError(f"frei_hip: {msg}")
            if len(hs) != nranks or any(len(x) != 64 for x in hs):
                raise RuntimeError("P2P setup failed on a peer rank (no mailbox handle)")
            # ranks on one GPU (the one-GPU rehearsal): no chained launches on this context
            # (every rank joins this exchange before any can fail in p2p_open)
            me = device_key(self.device).encode()
            if arg(me).count(me) > 1 and os.environ.get("FREI_CHAIN_SHARED") != "1":
                N.check(lib.frei_comm_shared_device(self._ctx, 1))
            allh = ctypes.create_string_buffer(b"".join(hs), 64 * nranks)
            N.check(lib.frei_comm_p2p_open(self._ctx, allh))
        elif kind == "host":
            def cb(send, recv, n, _user, _fn=arg, _R=nranks):
                try:
                    out = np.asarray(_fn(np.ctypeslib.as_array(send, (n,)).copy()),
                                     dtype=np.float64).ravel()
                    np.ctypeslib.as_array(recv, (_R * n,))[:] = out
                    return 0
                except Exception:  # surfaced as a C error, then RuntimeError
                    return 1
            self._ag_keep = N.ALLGATHER_FN(cb)
            N.check(lib.frei_comm_init_host(self._ctx, nranks, rank, self._ag_keep, None))
        else:
            raise ValueError(f"unknown comm kind {kind!r}")

    # ------------------------------------------------------------------ setup
    def _set_table(self, s, tab, sl):
        lib = N.lib()
        p, T = _table_arrays(tab)
        p_cgs, T = N.f64(p * BAR), N.f64(T)
        if isinstance(tab, BinnedTable):
            if tab.wavelength.size != self.lam_um.size:
                raise ValueError("binned table wavelengths must match the grid")
            N.check(lib.frei_set_table_binned(
                self._ctx, s, tab.xsec.handle(self.device), tab.mode, N.dptr(tab.wl_bins),
                N.dptr(tab.wavelength), tab.wavelength.size, self.lo, N.dptr(tab.temperature),
                tab.temperature.size, N.dptr(tab.pressure), tab.pressure.size))
            return
        if isinstance(tab, SeparableTable):
            N.check(lib.frei_set_table_separable(
                self._ctx, s, N.dptr(N.f64(tab.base[sl])), N.dptr(N.f64(tab.fp)),
                N.dptr(N.f64(tab.fT)), tab.lo, tab.hi, N.dptr(p_cgs), p.size, N.dptr(T), T.size))
            return
        vals = table_values(tab)      # transposed by name when the table carries .dims
        if vals.ndim != 3 or vals.shape[:2] != (p.size, T.size):
            raise ValueError("opacity table must be (pressure, temperature, wavelength)")
        if vals.shape[2] != self.lam_um.size:
            raise ValueError("opacity table wavelength axis must match the grid")
        v = N.f64(vals[:, :, sl])
        N.check(lib.frei_set_table(self._ctx, s, N.dptr(v), N.dptr(p_cgs), p.size,
                                   N.dptr(T), T.size))

    def close(self):
        if getattr(self, "_ctx", None):
            N.lib().frei_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ state
    def set_fluxes(self, up=None, down=None):
        N.check(N.lib().frei_set_fluxes(self._ctx, N.dptr(None if up is None else N.f64(up)),
                                        N.dptr(None if down is None else N.f64(down))))

    def get_fluxes(self):
        up = np.empty((self.n_layers, self.n_lam))
        down = np.empty((self.n_layers, self.n_lam))
        N.check(N.lib().frei_get_fluxes(self._ctx, N.dptr(up), N.dptr(down)))
        return up, down

    def get_spectrum(self):
        """The emergent spectrum F_up[-1] (core.py:335-338), one row read back."""
        spec = np.empty(self.n_lam)
        N.check(N.lib().frei_get_spectrum(self._ctx, N.dptr(spec)))
        return spec

    def set_temperatures(self, T):
        N.check(N.lib().frei_set_temperatures(self._ctx, N.dptr(N.f64(T))))

    def get_temperatures(self):
        T = np.empty(self.n_layers)
        N.check(N.lib().frei_get_temperatures(self._ctx, N.dptr(T)))
        return T

    # ------------------------------------------------------------------ compute
    def sweep(self, direction, alpha=1.0, want_dtaus=True):
        """One emit/absorb sweep on the device state -> (dT, bolometric[n_layers][4], dtaus)."""
        dT = np.empty(self.n_layers)
        bol = np.empty((self.n_layers, 4))
        dtaus = np.empty((self.n_layers, self.n_lam)) if want_dtaus else None
        N.check(N.lib().frei_sweep(self._ctx, direction, float(alpha), N.dptr(dT), N.dptr(bol),
                                   N.dptr(dtaus)))
        return dT, bol, dtaus

    def set_mmr(self, mmr):
        """Per-layer mass mixing ratios [n_species][n_layers] for the following sweeps."""
        self.mmr = N.f64(np.broadcast_to(np.asarray(mmr, dtype=float),
                                         (len(self.names), self.n_layers)))
        N.check(N.lib().frei_set_mmr(self._ctx, N.dptr(self.mmr)))

    def run(self, T_init, n_timesteps=1, n_zero_crossings=2, convergence_dT=3.0, alpha=1.0,
            want_dtaus=True):
        """Grid.emission_spectrum on the device (core.py:233-338)."""
        if self.provider is not None:
            return self._run_provider(T_init, n_timesteps, n_zero_crossings, convergence_dT,
                                      alpha, want_dtaus)
        nL = self.n_layers
        n_iter = ctypes.c_int(0)
        T_final = np.empty(nL)
        hist = np.empty(nL * 2 * n_timesteps)
        dtaus = np.empty((nL, self.n_lam)) if want_dtaus else None
        spec = np.empty(self.n_lam)
        N.check(N.lib().frei_run(self._ctx, N.dptr(N.f64(T_init)), int(n_timesteps),
                                 int(n_zero_crossings), float(convergence_dT), float(alpha),
                                 ctypes.byref(n_iter), N.dptr(T_final), N.dptr(hist),
                                 N.dptr(dtaus), N.dptr(spec)))
        it = n_iter.value
        temp_hist = hist[: nL * 2 * it].reshape(nL, 2 * it)
        return dict(spectrum=spec, final_T=T_final, temp_hist=temp_hist, dtaus=dtaus, n_iter=it)

    def _provider_step(self, T):
        """The provider's mixing ratios at every layer's (T, p), as kappa's chemistry call
        (opacity.py:246-248) sees them in the coming sweep."""
        self.set_mmr(provider_mmr(self.provider, T, self.p_bar, self.names, self.m_bar))

    def _run_provider(self, T_init, n_timesteps, n_zero_crossings, convergence_dT, alpha,
                      want_dtaus):
        """core.py:264-338 stepped from the host for a T-dependent chemistry provider: before
        every sweep the provider runs at the layers' current temperatures (read back from the
        device, 8 B per layer) and its mixing ratios go up; the sweeps, bolometric sums and T
        updates run on the device as in :meth:`run`.  The convergence test is core.py:301-318's
        (Q13) on the absorb sweeps' histories."""
        nL = self.n_layers
        self.state_init(T_init)              # zero fluxes (core.py:265-266), T = T_init
        T = self.get_temperatures()
        hists = []
        it = 0
        dT = np.empty(nL)
        for it in range(1, int(n_timesteps) + 1):
            self._provider_step(T)
            # (the loop reads back only what it uses: no bolometric sums, no emit dT)
            N.check(N.lib().frei_sweep(self._ctx, EMIT, float(alpha), None, None, None))
            T1 = self.get_temperatures()
            self._provider_step(T1)
            N.check(N.lib().frei_sweep(self._ctx, ABSORB, float(alpha), N.dptr(dT), None, None))
            T = self.get_temperatures()
            hists.append(np.stack([T1, T], axis=1))
            th = np.hstack(hists)
            th = th.T[th[0] != 0].T
            diffs = np.diff(th.T, axis=0)
            conv = ((np.count_nonzero(np.sign(diffs[1:]) != np.sign(diffs[:-1]), axis=0)
                     > n_zero_crossings) | (np.abs(dT) < convergence_dT))
            if np.all(conv):
                break
        self._provider_step(T)
        _, _, dtaus = self.sweep(EMIT, alpha=1.0, want_dtaus=want_dtaus)   # Q7: alpha = 1
        return dict(spectrum=self.get_spectrum(), final_T=self.get_temperatures(),
                    temp_hist=np.hstack(hists) if hists else np.empty((nL, 0)),
                    dtaus=dtaus, n_iter=it)

    def state_init(self, T_init):
        N.check(N.lib().frei_state_init(self._ctx, N.dptr(N.f64(T_init))))

    def iterate(self, n, n_zero_crossings=-1, convergence_dT=3.0, alpha=1.0):
        N.check(N.lib().frei_iterate(self._ctx, int(n), int(n_zero_crossings),
                                     float(convergence_dT), float(alpha)))

    def synchronize(self):
        N.check(N.lib().frei_synchronize(self._ctx))

    def timing(self, on):
        N.check(N.lib().frei_timing_enable(self._ctx, 1 if on else 0))

    def timing_read(self):
        ms = ctypes.c_double(0)
        n = ctypes.c_int(0)
        N.check(N.lib().frei_timing_read(self._ctx, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def timing_read_exchange(self):
        """(total ms, calls) of the timed rank exchanges (all-gathers) since timing(True)."""
        ms, n = ctypes.c_double(), ctypes.c_int()
        N.check(N.lib().frei_timing_read_exchange(self._ctx, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def milne_pressure(self, p_bar, dtaus=None):
        """Per-wavelength Milne pressures of this slice (core.py:392-395) from ``dtaus`` (host
        array) or, with None, the dtaus the last run left on the device."""
        out = np.empty(self.n_lam)
        d = None if dtaus is None else N.f64(dtaus)
        N.check(N.lib().frei_milne_pressure(self._ctx, N.dptr(d), N.dptr(N.f64(p_bar)),
                                            N.dptr(out)))
        return out

    def contribution(self, p_bar, T, dtaus=None):
        """Contribution function of this slice (plot.py:63-79), rows bottom-first."""
        p = np.asarray(p_bar, dtype=float)
        dlogP = (np.log10(p.max()) - np.log10(p.min())) / (len(p) - 1)
        k = 10 ** -dlogP
        ratio = N.f64(p / ((1 - k) * p))
        nu = N.f64(1.0 / (self.lam_um[self.lo:self.hi] * UM))
        cf = np.empty((self.n_layers, self.n_lam))
        d = None if dtaus is None else N.f64(dtaus)
        N.check(N.lib().frei_contribution(self._ctx, N.dptr(d), N.dptr(nu), N.dptr(ratio),
                                          N.dptr(N.f64(T)), H * C / K_B, N.dptr(cf)))
        return cf

    def path(self):
        """Sweep implementation the tables select: dict(fast, lds_steps, contracted, nan)."""
        f = ctypes.c_int(0)
        N.check(N.lib().frei_ctx_path(self._ctx, ctypes.byref(f)))
        v = f.value
        return dict(fast=bool(v & 1), lds_steps=bool(v & 2), contracted=bool(v & 4),
                    nan=bool(v & 8), paired=bool(v & 16), quad=bool(v & 32),
                    pipe=(v >> 6) & 7, lam2=bool(v & 512), tail=bool(v & 1024),
                    lazy_k3=bool(v & 2048))

    def set_option(self, name, value):
        """Tuning knob of include/frei_hip.h frei_set_option (e.g. "precontract", 0)."""
        N.check(N.lib().frei_set_option(self._ctx, name.encode(), int(value)))

    def graph_info(self):
        """(captures, replays) of the hipGraph T-P iteration replay (frei_graph_info)."""
        cap, rep = ctypes.c_int(0), ctypes.c_int(0)
        N.check(N.lib().frei_graph_info(self._ctx, ctypes.byref(cap), ctypes.byref(rep)))
        return cap.value, rep.value

    def tail_count(self):
        """Trailing-update launches so far (frei_tail_info): producer/consumer sweeps whose
        launch also ran their own fused update, layer by layer as the sweep published them."""
        n = ctypes.c_int64(0)
        N.check(N.lib().frei_tail_info(self._ctx, ctypes.byref(n)))
        return n.value

    def chain_count(self):
        """Chained sweep launches so far (frei_chain_info): sweeps whose launch also ran the
        previous sweep's deferred update."""
        n = ctypes.c_int64(0)
        N.check(N.lib().frei_chain_info(self._ctx, ctypes.byref(n)))
        return n.value

    def setup_timing(self):
        """Milliseconds of the last one-time metadata build by phase (frei_setup_timing)."""
        ms = np.zeros(5)
        N.check(N.lib().frei_setup_timing(self._ctx, N.dptr(ms)))
        return dict(zip(("brackets_host", "uploads", "eff_alloc", "eff_zero", "contract"),
                        ms.tolist()))

    def contract_timing(self):
        """The last species-contraction kernel (K3, or K7 for a batched context): dict(ms = its
        HIP-event duration, bytes = its algorithmic HBM bytes) (frei_contract_timing)."""
        ms, nb = ctypes.c_double(0), ctypes.c_double(0)
        N.check(N.lib().frei_contract_timing(self._ctx, ctypes.byref(ms), ctypes.byref(nb)))
        return dict(ms=ms.value, bytes=nb.value)

    def kappa(self, T, p_bar):
        k = np.empty(self.n_lam)
        sig = np.empty(self.n_lam)
        N.check(N.lib().frei_kappa(self._ctx, float(T), float(p_bar) * BAR, N.dptr(k),
                                   N.dptr(sig)))
        return k, sig


# ---------------------------------------------------------------------- shim engine cache
# The reference's seam functions (emit/absorb/kappa) are stateless and a caller may drive them
# in a Python loop, as Grid.emission_spectrum does (core.py:273-299).  A fresh context per
# call would re-upload every opacity table (30 GB at C3), so the shims keep the last few
# contexts, keyed on the identity of the opacity dict and its tables plus the grid arrays.
# Tables are treated as immutable while cached: after editing table values in place, call
# clear_engine_cache().
# [(key, (opacities, its tables) — kept alive so their ids stay unique while cached, engine)]
_ENGINE_CACHE = []
_ENGINE_CACHE_SIZE = 2


def _array_key(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=float))
    return (a.shape, hash(a.tobytes()))


def _tables_key(opacities):
    out = []
    for name, tab in opacities.items():
        vals = getattr(tab, "__dict__", {}).get("values")
        ptr = vals.ctypes.data if isinstance(vals, np.ndarray) else None
        out.append((name, id(tab), ptr))
    return (id(opacities), tuple(out))


def cached_engine(opacities, *, lam_um, p_bar, g, m_bar, F_toa, mmr=None, device=0,
                  chemistry=None, tag=None):
    """An :class:`Engine` for these tables and grid, reused across calls with the same
    opacity dict (by identity), equal grid arrays / scalars and the same chemistry provider
    (by identity); ``tag`` separates contexts whose mixing ratios a caller sets itself."""
    key = (_tables_key(opacities), _array_key(lam_um), _array_key(p_bar), float(g),
           float(m_bar), None if F_toa is None else _array_key(F_toa),
           None if mmr is None else _array_key(mmr), int(device),
           None if chemistry is None else id(chemistry), tag)
    for i, (k, _, eng) in enumerate(_ENGINE_CACHE):
        if k == key and eng._ctx:
            _ENGINE_CACHE.insert(0, _ENGINE_CACHE.pop(i))
            return eng
    eng = Engine(lam_um, p_bar, opacities, g=g, m_bar=m_bar, F_toa=F_toa, mmr=mmr,
                 device=device, chemistry=chemistry)
    # the provider is kept alive with the entry, so its id stays unique while cached
    _ENGINE_CACHE.insert(0, (key, (opacities, tuple(opacities.values()), chemistry, tag), eng))
    while len(_ENGINE_CACHE) > _ENGINE_CACHE_SIZE:
        _ENGINE_CACHE.pop()[2].close()
    return eng


def clear_engine_cache():
    """Release the contexts the emit/absorb/kappa shims keep between calls."""
    while _ENGINE_CACHE:
        _ENGINE_CACHE.pop()[2].close()


def propagate_fluxes_device(lam_um, F_1_up, F_2_down, T_1, T_2, delta_tau, omega_0, g_0=0.0,
                            device=0):
    """twostream.py:97-177 on the GPU; ``g_0`` scalar or per-wavelength (0: the call sites'
    value, twostream.py:389, 518)."""
    lam_cm = np.asarray(lam_um, dtype=float).ravel() * UM
    n = lam_cm.size
    bc = lambda a: N.f64(np.broadcast_to(np.asarray(a, dtype=float).ravel()
                                         if np.ndim(a) else a, (n,)))
    c1, lk = N.f64(planck_prefactor(lam_cm)), N.f64(lam_cm * K_B)
    F1u, F2d, dtau, w0 = bc(F_1_up), bc(F_2_down), bc(delta_tau), bc(omega_0)
    g0 = None if np.all(np.asarray(g_0) == 0) else bc(g_0)
    F2u, F1d = np.empty(n), np.empty(n)
    N.check(N.lib().frei_propagate_fluxes(device, n, N.dptr(c1), N.dptr(lk), N.dptr(F1u),
                                          N.dptr(F2d), float(T_1), float(T_2), N.dptr(dtau),
                                          N.dptr(w0), N.dptr(g0), N.dptr(F2u), N.dptr(F1d)))
    return F2u, F1d
