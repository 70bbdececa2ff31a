"""Determinism check of the batched (C5) path: the bench's C5 workload run to radiative
equilibrium three times in one process; prints per-run iteration counts and a hash of the
final temperatures and spectra.  With a third argument G > 0, G GiB of device memory are
first filled with 0xFF bytes (NaN doubles) and freed, so any read of memory the engine did not
initialise would show up as changed results.
With a fourth argument "afterc3", a C3 context is created, run and closed first (the bench's
order).
    python tools/c5_determinism.py [n_lam] [mh] [G] [afterc3]"""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from frei_amd.batch import BatchEngine          # noqa: E402
from frei_amd.opacity import SeparableTable     # noqa: E402
from frei_amd.tp import temperature_grid        # noqa: E402
from frei_amd.workloads import c3               # noqa: E402

n_lam = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
mh = float(sys.argv[2]) if len(sys.argv) > 2 else -1.0
dirty_gib = int(sys.argv[3]) if len(sys.argv) > 3 else 0
after_c3 = len(sys.argv) > 4 and sys.argv[4] == "afterc3"
if after_c3:   # the bench's order: a C3 context (30 GB of tables) created, iterated and closed first
    from frei_amd.engine import Engine
    w3 = c3()
    tabs3 = {n: SeparableTable(w3["base"][s], w3["fp"][s], w3["fT"][s], w3["p"], w3["T_nodes"])
             for s, n in enumerate(w3["names"])}
    e3 = Engine(w3["lam"], w3["p"], tabs3, mmr=w3["mmr"], device=0)
    e3.state_init(w3["T0"])
    e3.iterate(5)
    out3 = e3.run(w3["T0"], n_timesteps=50, n_zero_crossings=2, convergence_dT=3.0, want_dtaus=False)
    e3.close()
    del e3
    print(f"C3 context created, run ({out3['n_iter']} iterations) and closed", flush=True)
if dirty_gib > 0:
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipSetDevice(0)
    bufs = []
    for _ in range(dirty_gib // 8):   # 8 GiB pieces, all live at once, then freed
        b = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(b), ctypes.c_size_t(8 << 30)) == 0
        assert hip.hipMemset(b, 0xFF, ctypes.c_size_t(8 << 30)) == 0
        bufs.append(b)
    hip.hipDeviceSynchronize()
    for b in bufs:
        hip.hipFree(b)
    print(f"dirtied and freed {dirty_gib} GiB", flush=True)
w = c3(n_layers=60, n_lam=n_lam, n_T=16)
T_refs = np.arange(1000.0, 2401.0, 200.0)
loggs = np.array([2.5, 3.0, 3.5, 4.0])
T0 = np.array([temperature_grid(w["p"], t, 0.1, 0.1) for t in T_refs for _ in loggs])
g = np.array([10.0 ** lg for _ in T_refs for lg in loggs])
T_nodes = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 16)
fT = (T_nodes / 1000.0) ** 0.5
tabs = {n: SeparableTable(w["base"][s], w["fp"][s], fT, w["p"], T_nodes)
        for s, n in enumerate(w["names"])}
mmr = np.broadcast_to(w["mmr"] * 10.0 ** mh, (len(g),) + w["mmr"].shape)
eng = BatchEngine(w["lam"], w["p"], tabs, g=g, mmr=mmr, device=0)
try:
    eng.state_init(T0)
    eng.iterate(6)
    for r in range(3):
        out = eng.run(T0, n_timesteps=200, n_zero_crossings=2, convergence_dT=3.0)
        h = hashlib.sha1(out["final_T"].tobytes() + out["spectra"].tobytes()).hexdigest()[:12]
        print(f"run {r}: n_iter {out['n_iter'].tolist()} hash {h}", flush=True)
finally:
    eng.close()
