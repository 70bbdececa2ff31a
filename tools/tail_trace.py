"""Where a trailing-update launch's time goes (FREI_TRACE build, round 6).

    FREI_HIP_LIB=trace_build/trace.so python tools/tail_trace.py [--n-lam 62500] [--tail 1]

Records (frei_kernels.hip TRACE_*): sweep blocks of sweep_pipe_tail_kernel (kind 64: entry, end
of prologue, end of the phase loop, exit) and the update body (kind 30; thread 0 of each
trailing block, i.e. slot 0 of every round: entry, partial sums landed, dT published, exit).
Per launch, relative to its first sweep-block entry (medians over launches): sweep entries,
last loop end, last exit, every update round's entry / sums landed / exit, the next launch's
first entry."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-lam", type=int, default=62500)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tail", type=int, default=1)
    a = ap.parse_args()
    from frei_amd import _native as N
    from frei_amd.engine import Engine
    from frei_amd.opacity import SeparableTable
    from frei_amd.workloads import c3
    w = c3(n_lam=a.n_lam, species=None)
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, n in enumerate(w["names"])}
    eng = Engine(w["lam"], w["p"], tabs, mmr=w["mmr"], device=0)
    eng.set_option("tail", a.tail)
    print("path", eng.path())
    L = N.lib()
    fetch = L.frei_trace_fetch
    fetch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    cap = 1 << 17
    buf = np.zeros((cap, 8), dtype=np.int64)
    n = ctypes.c_int(0)
    eng.state_init(w["T0"])
    eng.iterate(3)
    eng.synchronize()
    fetch(buf.ctypes.data, cap, ctypes.byref(n))
    import time
    t0 = time.perf_counter()
    eng.iterate(a.iters)
    eng.synchronize()
    wall = (time.perf_counter() - t0) / a.iters * 1e6
    N.check(fetch(buf.ctypes.data, cap, ctypes.byref(n)))
    rec = buf[:min(n.value, cap)].copy()
    tick = 0.01
    print(f"{a.iters} iterations, {wall:.1f} us each (wall); {len(rec)} records; kinds "
          f"{sorted(set(int(k) for k in rec[:, 0]))}")
    sw = rec[(rec[:, 0] != 30) & (rec[:, 0] != 31)]
    up = rec[(rec[:, 0] == 30) | (rec[:, 0] == 31)]
    # launches: sweep records grouped by entry time (a new launch starts after the previous
    # launch's last sweep exit)
    sw = sw[np.argsort(sw[:, 2])]
    groups, cur, end = [], [], None
    for r in sw:
        if end is not None and r[2] > end:
            groups.append(np.array(cur))
            cur, end = [], None
        cur.append(r)
        end = r[5] if end is None else max(end, r[5])
    groups.append(np.array(cur))
    rows = []
    for i, g in enumerate(groups[:-1]):
        t = g[:, 2].min()
        t_next = groups[i + 1][:, 2].min()
        u = up[(up[:, 2] >= t) & (up[:, 2] < t_next)]
        u = u[np.argsort(u[:, 2])]
        rows.append(dict(entry_spread=(g[:, 2].max() - t) * tick,
                         pro_end=(np.median(g[:, 3]) - t) * tick,
                         pro_end_max=(g[:, 3].max() - t) * tick,
                         loop_end_max=(g[:, 4].max() - t) * tick,
                         exit_max=(g[:, 5].max() - t) * tick,
                         next_entry=(t_next - t) * tick,
                         upd=[((x[2] - t) * tick,
                               (((x[2] >> 40) << 40 | (x[3] & ((1 << 40) - 1))) - t) * tick,
                               (x[4] - t) * tick, (x[5] - t) * tick, int(x[1]), int(x[3] >> 40))
                              for x in u]))
    for k in ("entry_spread", "pro_end", "pro_end_max", "loop_end_max", "exit_max", "next_entry"):
        print(f"  {k:>14s}: median {np.median([r[k] for r in rows]):7.2f} us")
    if rows and rows[len(rows) // 2]["upd"]:
        print("  update rounds of one launch (entry, slot 0's last poll done, all slots' sums "
              "summed, exit, block, poll passes):")
        for x in rows[len(rows) // 2]["upd"]:
            print(f"     {x[0]:7.2f} {x[1]:7.2f} {x[2]:7.2f} {x[3]:7.2f}  b{x[4]}  {x[5]}")
    eng.close()


if __name__ == "__main__":
    main()
