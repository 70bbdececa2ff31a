"""Per-rank sweep time of the N-GPU split at the GLOBAL temperatures.

    python tools/slice_globalT.py [--n 8] [--iters 40]

A one-rank run of one slice (tools/projection.sh) evolves its temperatures from that slice's
bolometric sums alone, so late in the run each slice sweeps a different atmosphere than it would
as one rank of an N-GPU run (where every rank shares the global T).  Here the full 500k problem
runs `iters` T-P iterations on one GPU; its temperatures are then given to every slice's engine,
whose sweeps (emit and absorb, HIP events on the engine's stream) are timed at those
temperatures — the sweep cost each rank would have.  Also printed: the same slices at the initial
temperatures.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sweep_ms(eng, T, reps=6):
    ms = []
    for _ in range(reps):
        eng.set_temperatures(T)
        eng.timing(True)
        eng.sweep(0, alpha=1.0)
        eng.sweep(1, alpha=1.0)
        eng.synchronize()
        t, n = eng.timing_read()
        eng.timing(False)
        ms.append(t / max(n, 1))
    return float(np.median(ms[1:]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    from frei_amd.engine import Engine, partition
    from frei_amd.opacity import SeparableTable
    from frei_amd.workloads import c3
    w = c3(n_lam=500_000)
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, n in enumerate(w["names"])}
    full = Engine(w["lam"], w["p"], tabs, mmr=w["mmr"], device=0)
    full.state_init(w["T0"])
    full.iterate(a.iters, n_zero_crossings=10 ** 6, convergence_dT=-1.0)
    full.synchronize()
    Tg = full.get_temperatures()
    full.close()
    print(f"global T after {a.iters} iterations: {Tg.min():.1f}..{Tg.max():.1f} K")
    for r in range(a.n):
        lo, hi = partition(500_000, a.n, r)
        eng = Engine(w["lam"], w["p"], tabs, mmr=w["mmr"], device=0, lam_slice=(lo, hi))
        eng.state_init(w["T0"])
        t0 = sweep_ms(eng, w["T0"])
        tg = sweep_ms(eng, Tg)
        path = eng.path()
        eng.close()
        print(f"slice {r}/{a.n} [{lo}, {hi}): sweep {t0 * 1e3:.2f} us at T0, {tg * 1e3:.2f} us at the "
              f"global T (pipe {path.get('pipe')}, paired {path.get('paired')})")


if __name__ == "__main__":
    main()
