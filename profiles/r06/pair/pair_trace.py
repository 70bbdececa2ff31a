"""Where a paired trailing-update launch's time goes (FREI_TRACE build, round 6).

    FREI_HIP_LIB=trace_build/trace.so python tools/pair_trace.py [--pair 1]

Sweep-block records of the trailing-update kernels (kind 64: emit, 164: absorb; marks: body
entry, phase 0 published, loop end, exit) of 20 T-P iterations at the 8-GPU slice.  Per
iteration, relative to the first emit block's entry (medians over iterations): emit phase-0
publish / loop end (slowest block), absorb entry / phase-0 publish / loop end, next emit entry."""
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
    ap.add_argument("--iters", type=int, default=20)
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
    print("path", eng.path())
    fetch = N.lib().frei_trace_fetch
    fetch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    cap = 1 << 17
    buf = np.zeros((cap, 8), dtype=np.int64)
    n = ctypes.c_int(0)
    eng.state_init(w["T0"])
    eng.iterate(3)
    eng.synchronize()
    fetch(buf.ctypes.data, cap, ctypes.byref(n))
    eng.iterate(a.iters)
    eng.synchronize()
    N.check(fetch(buf.ctypes.data, cap, ctypes.byref(n)))
    rec = buf[:min(n.value, cap)]
    tick = 0.01
    em = rec[rec[:, 0] == 64]
    ab = rec[rec[:, 0] == 164]
    em = em[np.argsort(em[:, 2])]
    # iterations: emit records grouped by entry gaps (> 20 us between consecutive entries)
    starts = [0] + [i for i in range(1, len(em)) if em[i, 2] - em[i - 1, 2] > 2000]
    rows = []
    for g, s0 in enumerate(starts[:-1]):
        e = em[s0:starts[g + 1]]
        t0 = e[:, 2].min()
        t_next = em[starts[g + 1], 2]
        b = ab[(ab[:, 2] >= t0) & (ab[:, 2] < t_next)]
        if len(b) == 0:
            continue
        rows.append(dict(em_pro=(np.median(e[:, 3]) - t0) * tick,
                         em_loop_end=(e[:, 4].max() - t0) * tick,
                         ab_entry=(np.median(b[:, 2]) - t0) * tick,
                         ab_pro=(np.median(b[:, 3]) - t0) * tick,
                         ab_pro_max=(b[:, 3].max() - t0) * tick,
                         ab_loop_end=(b[:, 4].max() - t0) * tick,
                         next_emit=(t_next - t0) * tick))
    print(f"{len(rows)} iterations with both sweeps")
    # one middle iteration's update slots (kind 31: entry, last poll done, sums, exit; us)
    up = rec[rec[:, 0] == 31]
    g = len(starts) // 2
    t0 = em[starts[g], 2]
    t1 = em[starts[g + 1], 2] if g + 1 < len(starts) else t0 + 10 ** 9
    u = up[(up[:, 2] >= t0) & (up[:, 2] < t1)]
    u = u[np.argsort(u[:, 2])]
    print("  update rounds of the middle iteration (entry, last poll done, sums, exit, block):")
    for x in u:
        done = ((x[2] >> 40) << 40 | (x[3] & ((1 << 40) - 1)))
        print(f"     {(x[2] - t0) * tick:7.2f} {(done - t0) * tick:7.2f} {(x[4] - t0) * tick:7.2f} "
              f"{(x[5] - t0) * tick:7.2f}  b{int(x[1])}")
    for k in ("em_pro", "em_loop_end", "ab_entry", "ab_pro", "ab_pro_max", "ab_loop_end",
              "next_emit"):
        print(f"  {k:>12s}: median {np.median([r[k] for r in rows]):7.2f} us")
    eng.close()


if __name__ == "__main__":
    main()
