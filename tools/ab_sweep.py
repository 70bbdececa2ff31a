"""A/B timing of sweep-kernel builds (same C ABI) interleaved in ONE process.

    python tools/ab_sweep.py NAME=path/to/lib.so[:Q] [NAME=...] [--n-lam N] [--rounds R]

A ":Q" suffix forces Q lanes per wavelength (FREI_GROUP_Q) for that context.

Each library gets its own context on device 0 with the C3 workload; rounds alternate
between builds (MI355X guide §5.4 rule 24) and report median / min ms per sweep.
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    args = [a for a in sys.argv[1:] if "=" in a and not a.startswith("--")]
    opts = dict(a.lstrip("-").split("=") for a in sys.argv[1:] if a.startswith("--"))
    n_lam = int(opts.get("n-lam", 500_000))
    rounds = int(opts.get("rounds", 5))
    iters = int(opts.get("iters", 4))
    S = int(opts.get("species", 8))
    import importlib
    from frei_amd import _native as N
    from frei_amd.workloads import c3
    w = c3(n_lam=n_lam, species=None)
    names = w["names"][:S]
    builds = []
    for a in args:
        name, path = a.split("=", 1)
        env = {}
        if "@" in path:   # NAME=lib.so@VAR=v,VAR2=w: environment while the context is created
            path, spec = path.split("@", 1)
            env = dict(kv.split("=", 1) for kv in spec.split(","))
        q = None
        if ":" in path:
            path, q = path.rsplit(":", 1)
        N._lib = None
        N.LIB_PATH = os.path.abspath(path)
        lib = N.lib()
        import frei_amd.engine as E
        importlib.reload(E)
        from frei_amd.opacity import SeparableTable
        tabs = {n: SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
                for s, n in enumerate(names)}
        if q is not None:
            os.environ["FREI_GROUP_Q"] = q
        os.environ.update(env)
        eng = E.Engine(w["lam"], w["p"], tabs, mmr=w["mmr"][:S], device=0)
        os.environ.pop("FREI_GROUP_Q", None)
        for k in env:
            os.environ.pop(k, None)
        eng.state_init(w["T0"])
        eng.iterate(1)
        eng.synchronize()
        builds.append((name, lib, eng, []))
    res_it = {}
    for r in range(rounds):
        for name, lib, eng, res in builds:
            N._lib = lib
            eng.timing(True)
            t0 = time.perf_counter()
            eng.iterate(iters)
            eng.synchronize()
            res_it.setdefault(name, []).append((time.perf_counter() - t0) * 1e3 / iters)
            ms, n = eng.timing_read()
            eng.timing(False)
            res.append(ms / n)
    bpu = 8 + 16 + 16 * S
    for name, lib, eng, res in builds:
        med = float(np.median(res))
        print(f"{name:>14s}: sweep median {med:.4f} ms  min {min(res):.4f} ms  "
              f"{bpu * (w['p'].size - 1) * n_lam / (min(res) * 1e-3) / 1e12:.3f} TB/s algorithmic "
              f"({n_lam} lambda, {S} species); T-P iteration median "
              f"{float(np.median(res_it[name])):.4f} ms (wall, {iters} per round)")
    for name, lib, eng, res in builds:   # close every context with its own library
        N._lib = lib
        eng.close()


if __name__ == "__main__":
    main()
