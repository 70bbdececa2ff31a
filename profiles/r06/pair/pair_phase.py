"""Paired launch at the 8-GPU slice, per-wave stamps (FREI_TRACE build; PT_STAMP): for the
absorb sweep of the last iteration, per sampled block (shader cycles, relative to that block's
last emit barrier release): step records in LDS, loop start, phase 0 barrier arrival / release.

    FREI_HIP_LIB=trace_build/trace.so python tools/pair_phase.py [--pair 1]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pair", type=int, default=1)
    a = ap.parse_args()
    from frei_amd import _native as N
    from frei_amd.engine import Engine
    from frei_amd.opacity import SeparableTable
    from frei_amd.workloads import c3
    w = c3(n_lam=62500, species=None)
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, n in enumerate(w["names"])}
    eng = Engine(w["lam"], w["p"], tabs, mmr=w["mmr"], device=0)
    eng.set_option("tail_pair", a.pair)
    fetch = N.lib().frei_ptrace_fetch
    fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(2 * 8 * 16 * 25 * 2, dtype=np.int64)
    eng.state_init(w["T0"])
    eng.iterate(6)
    eng.synchronize()
    assert fetch(buf.ctypes.data, buf.size) == buf.size
    t = buf.reshape(2, 8, 16, 25, 2)
    nph = int(np.max(np.nonzero(t[0, 0, 0, :, 0])[0]))
    rows = []
    for b in range(8):
        if t[1, b, 0, 0, 0] == 0:
            continue
        ref = t[0, b, :, nph, 1].max()          # the block's last emit barrier release
        rec = t[1, b, :, 0, 1].max() - ref      # step records in LDS (slowest wave)
        start = t[1, b, :, 0, 0].max() - ref    # loop start (slowest wave)
        arr0 = t[1, b, :, 1, 0].max() - ref     # phase 0 barrier: last arrival
        rel0 = t[1, b, :, 1, 1].max() - ref
        rows.append((rec, start, arr0, rel0))
    r = np.array(rows)
    print(f"pair {a.pair}: absorb after the block's last emit barrier (cycles, median over "
          f"{len(r)} blocks): records {np.median(r[:, 0]):.0f}, loop start {np.median(r[:, 1]):.0f}, "
          f"phase 0 last arrival {np.median(r[:, 2]):.0f}, release {np.median(r[:, 3]):.0f}")
    eng.close()


if __name__ == "__main__":
    main()
