"""Where a T-P half-iteration's time goes, from in-kernel wall-clock marks (FREI_TRACE build).

    FREI_HIP_LIB=abv/trace.so python tools/trace_probe.py [--n-lam 62500] [--p2p] [--iters 40]

Every block of the sweeps and of the fused update records (kind, block, entry, end of
prologue, end of main loop, exit) at 100 MHz (frei_kernels.hip, FREI_TRACE).  Records are
grouped into launches (kernels on one stream never overlap), and per kind the medians over
launches are printed: the gap from the previous launch's last exit to this launch's first
entry, the spread of block entries, and per block the prologue, loop and epilogue.  The
half-iteration is a sweep's first entry to the next sweep's first entry.
"""
import argparse
import ctypes
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KIND = {1: "sweep_fast", 2: "sweep_pair", 12: "sweep_group2", 14: "sweep_group4", 21: "sweep_pipe1",
        22: "sweep_pipe2", 24: "sweep_pipe4", 30: "update_fused", 42: "chain_group2",
        44: "chain_group4", 41: "chain_fast", 54: "chain_pipe4"}


def chained(rec, tick):
    """Launches by time overlap (a chained launch holds update and sweep blocks): per kind, the
    medians over launches of the first entry, median prologue end, last loop end and last exit,
    all relative to the launch's first entry."""
    rec = rec[np.argsort(rec[:, 2], kind="stable")]
    cl, cur_end = [], None
    for r in rec:
        if cur_end is None or r[2] > cur_end:
            cl.append([])
            cur_end = r[5]
        cl[-1].append(r)
        cur_end = max(cur_end, r[5])
    by = {}
    for i, c in enumerate(cl):
        a = np.array(c)
        t0 = a[:, 2].min()
        key = tuple(sorted({int(k) for k in a[:, 0]}))
        row = {}
        for k in key:
            b = a[a[:, 0] == k]
            row[k] = ((b[:, 2].min() - t0) * tick, (np.median(b[:, 3]) - t0) * tick,
                      (b[:, 4].max() - t0) * tick, (b[:, 5].max() - t0) * tick)
        gap = (t0 - cl[i - 1][-1][5]) * tick if i else None
        prev_end = max(x[5] for x in cl[i - 1]) if i else None
        by.setdefault(key, []).append((row, (t0 - prev_end) * tick if i else None,
                                       (a[:, 5].max() - t0) * tick))
    for key, rows in by.items():
        print(f"launch type {[KIND.get(k, k) for k in key]}: {len(rows)} launches; median gap from "
              f"previous launch {np.median([g for _, g, _ in rows if g is not None]):.2f} us, "
              f"span {np.median([s for _, _, s in rows]):.2f} us")
        for k in key:
            v = np.median(np.array([r[k] for r, _, _ in rows]), axis=0)
            print(f"   {KIND.get(k, k):>14s}: first entry {v[0]:6.2f}  median prologue end {v[1]:6.2f}"
                  f"  last loop end {v[2]:6.2f}  last exit {v[3]:6.2f}")


def launches(rec):
    rec = rec[np.argsort(rec[:, 2], kind="stable")]
    out, cur, cur_end = [], None, None
    for r in rec:
        k = int(r[0])
        if cur is None or k != cur["kind"] or r[2] > cur_end:
            cur = {"kind": k, "rows": []}
            out.append(cur)
            cur_end = r[5]
        cur["rows"].append(r)
        cur_end = max(cur_end, r[5])
    for L in out:
        a = np.array(L["rows"])
        L["start"], L["end"] = int(a[:, 2].min()), int(a[:, 5].max())
        L["spread"] = int(a[:, 2].max() - a[:, 2].min())
        L["pro"] = float(np.median(a[:, 3] - a[:, 2]))
        L["loop"] = float(np.median(a[:, 4] - a[:, 3]))
        L["epi"] = float(np.median(a[:, 5] - a[:, 4]))
        L["last_loop_end"] = int(a[:, 4].max())
        L["n"] = len(a)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-lam", type=int, default=62500)
    ap.add_argument("--p2p", action="store_true", help="one-rank P2P exchange (bench --force-comm)")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--slice", default=None,
                    help="R/N: rank R's slice of an N-way partition of the --n-lam grid")
    ap.add_argument("--blocks", action="store_true", help="per-block loop-time distribution")
    a = ap.parse_args()
    from frei_amd import _native as N
    from frei_amd.engine import Engine
    from frei_amd.opacity import SeparableTable
    from frei_amd.workloads import c3
    w = c3(n_lam=a.n_lam, species=None)
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, n in enumerate(w["names"])}
    comm = None
    if a.p2p:
        from frei_amd.distributed import p2p_comm
        from frei_amd.rendezvous import Rendezvous
        comm = p2p_comm(Rendezvous(1, 0))
    kw = {}
    if a.slice:
        from frei_amd.engine import partition
        r, nr = (int(x) for x in a.slice.split("/"))
        kw["lam_slice"] = partition(a.n_lam, nr, r)
    eng = Engine(w["lam"], w["p"], tabs, mmr=w["mmr"], device=0, comm=comm, **kw)
    L = N.lib()
    if not hasattr(L, "frei_trace_fetch"):   # a production build: the wall-clock rate only
        eng.state_init(w["T0"])
        eng.iterate(a.warmup)
        eng.synchronize()
        walls = []
        for _ in range(5):
            t0 = time.perf_counter()
            eng.iterate(a.iters)
            eng.synchronize()
            walls.append((time.perf_counter() - t0) / a.iters * 1e3)
        print(f"slice {a.slice} {kw.get('lam_slice')}  n_lam {a.n_lam}  p2p {a.p2p}: "
              f"{np.median(walls) * 1e3:.2f} us per T-P iteration (median of 5 x {a.iters}; "
              f"min {min(walls) * 1e3:.2f})")
        eng.close()
        return
    fetch = L.frei_trace_fetch
    fetch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    cap = 1 << 17
    buf = np.zeros((cap, 8), dtype=np.int64)   # kind, block, 4 wall marks, 2 cycle stamps
    n = ctypes.c_int(0)
    eng.state_init(w["T0"])
    eng.iterate(a.warmup)
    eng.synchronize()
    fetch(buf.ctypes.data, cap, ctypes.byref(n))
    t0 = time.perf_counter()
    eng.iterate(a.iters)
    eng.synchronize()
    wall = (time.perf_counter() - t0) / a.iters * 1e3
    N.check(fetch(buf.ctypes.data, cap, ctypes.byref(n)))
    if n.value > cap:
        print(f"trace overflow: {n.value} records > {cap}")
    rec = buf[:min(n.value, cap)].copy()
    tick = 0.01   # us per wall_clock64 tick (100 MHz)
    if any(int(k) >= 40 for k in rec[:, 0]):
        print(f"slice {a.slice}  n_lam {a.n_lam}  p2p {a.p2p}  {a.iters} T-P iterations: "
              f"{wall * 1e3:.2f} us each (wall, no profiler)")
        chained(rec, tick)
        eng.close()
        return
    Ls = launches(rec)
    for i in range(1, len(Ls)):
        Ls[i]["gap"] = (Ls[i]["start"] - Ls[i - 1]["end"]) * tick
    Ls[0]["gap"] = None
    kinds = sorted({L_["kind"] for L_ in Ls})
    print(f"slice {a.slice} {kw.get('lam_slice')}  n_lam {a.n_lam}  p2p {a.p2p}  {a.iters} T-P iterations: {wall * 1e3:.2f} us each "
          f"(wall, no profiler); {len(Ls)} launches")
    print(f"{'kind':>14s} {'n':>4s} {'blocks':>6s} {'gap_in':>7s} {'spread':>7s} {'prolog':>7s} "
          f"{'loop':>7s} {'epilog':>7s} {'span':>7s} {'tail':>7s}   (median us)")
    for k in kinds:
        sel = [L_ for L_ in Ls if L_["kind"] == k]
        med = lambda f: statistics.median([f(L_) for L_ in sel])
        gaps = [L_["gap"] for L_ in sel if L_["gap"] is not None]
        print(f"{KIND.get(k, k):>14s} {len(sel):4d} {sel[0]['n']:6d} "
              f"{statistics.median(gaps) if gaps else float('nan'):7.2f} "
              f"{med(lambda x: x['spread']) * tick:7.2f} {med(lambda x: x['pro']) * tick:7.2f} "
              f"{med(lambda x: x['loop']) * tick:7.2f} {med(lambda x: x['epi']) * tick:7.2f} "
              f"{med(lambda x: x['end'] - x['start']) * tick:7.2f} "
              f"{med(lambda x: x['end'] - x['last_loop_end']) * tick:7.2f}")
    sw = [L_ for L_ in Ls if KIND.get(L_["kind"], "").startswith("sweep")]
    if a.blocks and sw:
        # per block: loop time and exit relative to the launch's first entry, medians over launches
        nb = max(len(L_["rows"]) for L_ in sw)
        loop = np.full((len(sw), nb), np.nan)
        ex = np.full((len(sw), nb), np.nan)
        for i, L_ in enumerate(sw):
            for r in L_["rows"]:
                loop[i, r[1]] = (r[4] - r[3]) * tick
                ex[i, r[1]] = (r[5] - L_["start"]) * tick
        lm, em = np.nanmedian(loop, axis=0), np.nanmedian(ex, axis=0)
        q = np.percentile(lm, [0, 10, 50, 90, 99, 100])
        print("sweep block loop time percentiles (0,10,50,90,99,100):", np.round(q, 2))
        q = np.percentile(em, [0, 10, 50, 90, 99, 100])
        print("sweep block exit time percentiles (0,10,50,90,99,100):", np.round(q, 2))
        nbin = 16
        edges = np.linspace(0, nb, nbin + 1).astype(int)
        print("by block index (16 bins): loop mean / exit max")
        print(" ".join(f"{np.mean(lm[edges[i]:edges[i+1]]):.1f}/{np.max(em[edges[i]:edges[i+1]]):.1f}"
                       for i in range(nbin)))
        slow = np.argsort(em)[-8:]
        print("slowest blocks:", [(int(b), round(float(em[b]), 2), round(float(lm[b]), 2)) for b in slow])
    halves = [(sw[i + 1]["start"] - sw[i]["start"]) * tick for i in range(len(sw) - 1)]
    if halves:
        print(f"half-iteration (sweep entry to next sweep entry): median {statistics.median(halves):.2f} us")
    eng.close()


if __name__ == "__main__":
    main()
