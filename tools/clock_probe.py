"""Shader clock of the T-P loop over time, from in-kernel stamps (FREI_TRACE build).

    FREI_HIP_LIB=abtree/trace.so python tools/clock_probe.py [--n-lam 500000] [--chunks 12]
        [--chunk-iters 5] [--soak-s 3]

Every block of the sweeps and of the fused update stamps the wall clock (s_memrealtime,
100 MHz) and the shader-cycle counter (s_memtime) at entry and exit (frei_kernels.hip,
FREI_TRACE); cycles / wall x 100 MHz is the clock that block ran at (MI355X_MICROARCH.md,
DVFS item 6).  The probe runs the bench's workload (C3, contracted table) from state_init in
chunks of a few T-P iterations, the first chunks covering bench.py's warm-up + timed window
(3 + 20 iterations), then soaks the GPU for --soak-s seconds of back-to-back iterations and
reads a last chunk: per chunk the wall time per iteration and the median clock of the sweep
and update blocks.  Diagnostic build only: its stamps cost a few per cent, so read the clock
and the shares, not the build's run time.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-lam", type=int, default=500_000)
    ap.add_argument("--chunks", type=int, default=12)
    ap.add_argument("--chunk-iters", type=int, default=5)
    ap.add_argument("--soak-s", type=float, default=3.0)
    a = ap.parse_args()
    from frei_amd import _native as N
    from frei_amd.engine import Engine
    from frei_amd.opacity import SeparableTable
    from frei_amd.workloads import c3
    w = c3(n_lam=a.n_lam)
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, n in enumerate(w["names"])}
    eng = Engine(w["lam"], w["p"], tabs, mmr=w["mmr"], device=0)
    L = N.lib()
    if not hasattr(L, "frei_trace_fetch"):
        raise SystemExit("needs a FREI_TRACE build (FREI_HIP_LIB=...)")
    fetch = L.frei_trace_fetch
    fetch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    cap = 1 << 17
    buf = np.zeros((cap, 8), dtype=np.int64)
    n = ctypes.c_int(0)
    eng.path()
    eng.state_init(w["T0"])
    eng.synchronize()
    N.check(fetch(buf.ctypes.data, cap, ctypes.byref(n)))

    def chunk(label, it0):
        t0 = time.perf_counter()
        eng.iterate(a.chunk_iters)
        eng.synchronize()
        wall = (time.perf_counter() - t0) / a.chunk_iters * 1e6
        N.check(fetch(buf.ctypes.data, cap, ctypes.byref(n)))
        rec = buf[:min(n.value, cap)]
        dt = (rec[:, 5] - rec[:, 2]).astype(float)
        ok = dt > 0
        ghz = (rec[:, 7] - rec[:, 6])[ok] / dt[ok] * 0.1   # cycles per 10 ns -> GHz
        kind = rec[ok, 0]
        sweep = ghz[kind < 30]
        upd = ghz[kind == 30]
        print(f"{label:>18s} iters {it0:5d}-{it0 + a.chunk_iters - 1:5d}: {wall:8.1f} us/iter  "
              f"sweep clock median {np.median(sweep) if sweep.size else float('nan'):.3f} GHz "
              f"(p10 {np.percentile(sweep, 10) if sweep.size else float('nan'):.3f}, "
              f"p90 {np.percentile(sweep, 90) if sweep.size else float('nan'):.3f})  "
              f"update clock median {np.median(upd) if upd.size else float('nan'):.3f} GHz  "
              f"records {n.value}", flush=True)

    it = 0
    for c in range(a.chunks):
        chunk("from state_init", it)
        it += a.chunk_iters
    t_end = time.perf_counter() + a.soak_s
    soaked = 0
    while time.perf_counter() < t_end:
        eng.iterate(20)
        eng.synchronize()
        soaked += 20
    N.check(fetch(buf.ctypes.data, cap, ctypes.byref(n)))
    it += soaked
    for c in range(3):
        chunk(f"after {a.soak_s:.0f} s soak", it)
        it += a.chunk_iters
    eng.close()


if __name__ == "__main__":
    main()
