"""Per-phase timeline of the producer/consumer sweep (FREI_TRACE build).

    FREI_HIP_LIB=trace_build/trace.so python tools/pipe_trace.py [--n-lam 62500]

Lane 0 of every wave of 8 sampled blocks stamps the shader-cycle counter at the loop start and,
per phase, on reaching and on leaving the block barrier (frei_kernels.hip PT_STAMP; the last
launch per direction).  Printed per direction and phase, medians over the sampled blocks, in
shader cycles: the phase length (barrier release to release), per role the work before the
barrier (previous release -> arrival) and the wait in it (arrival -> release), and which role
arrived last."""
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
    a = ap.parse_args()
    from frei_amd import _native as N
    from frei_amd.engine import Engine
    from frei_amd.opacity import SeparableTable
    from frei_amd.workloads import c3
    w = c3(n_lam=a.n_lam, species=None)
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, n in enumerate(w["names"])}
    eng = Engine(w["lam"], w["p"], tabs, mmr=w["mmr"], device=0)
    eng.set_option("tail", 0)
    print("path", eng.path())
    L = N.lib()
    fetch = L.frei_ptrace_fetch
    fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nph_cap = 24
    buf = np.zeros(2 * 8 * 16 * (nph_cap + 1) * 2, dtype=np.int64)
    eng.state_init(w["T0"])
    eng.iterate(a.iters)
    eng.synchronize()
    assert fetch(buf.ctypes.data, buf.size) == buf.size
    t = buf.reshape(2, 8, 16, nph_cap + 1, 2)
    nph = int(np.max(np.nonzero(t[0, 0, 0, :, 0])[0]))   # last stamped phase index (+1 offset)
    roles = [((wv + (wv >> 2)) & 3) for wv in range(16)]
    for d in (0, 1):
        blocks = [b for b in range(8) if t[d, b, 0, 0, 0] != 0]
        print(f"dir {d}: {len(blocks)} sampled blocks, {nph} barriers")
        print("  ph   length | prod work  wait | cons work  wait | last (P/C)")
        tot = []
        for k in range(1, nph + 1):
            L_, pw, pwt, cw, cwt, last = [], [], [], [], [], []
            for b in blocks:
                rel_prev = np.max(t[d, b, :, k - 1, 1]) if k > 1 else None
                start = t[d, b, :, 0, 0] if k == 1 else t[d, b, :, k - 1, 1]
                arr = t[d, b, :, k, 0]
                rel = t[d, b, :, k, 1]
                if k > 1:
                    L_.append(np.max(rel) - rel_prev)
                work = arr - start
                wait = rel - arr
                for wv in range(16):
                    (cw if roles[wv] == 3 else pw).append(work[wv])
                    (cwt if roles[wv] == 3 else pwt).append(wait[wv])
                last.append("C" if roles[int(np.argmax(arr))] == 3 else "P")
            lm = np.median(L_) if L_ else float("nan")
            tot.append(lm)
            print(f"  {k - 1:2d} {lm:8.0f} | {np.median(pw):8.0f} {np.median(pwt):5.0f} | "
                  f"{np.median(cw):8.0f} {np.median(cwt):5.0f} | "
                  f"{last.count('P')}/{last.count('C')}")
        # per SIMD (waves w, w + 4, w + 8, w + 12), phases 1 .. nph - 2: arrival order of its four
        # waves after the previous release, with the role of each
        order = {}
        for b in blocks:
            for k in range(2, nph - 1):
                rel_prev = np.max(t[d, b, :, k - 1, 1])
                for simd in range(4):
                    ws = [simd + 4 * q for q in range(4)]
                    arr = sorted((t[d, b, wv, k, 0] - rel_prev, roles[wv]) for wv in ws)
                    for r, (x, role) in enumerate(arr):
                        order.setdefault(r, []).append((x, role))
        print("  per SIMD, arrival rank: median cycles after the previous release, roles "
              "(P0 P1 P2 C counts)")
        for r in sorted(order):
            xs = [x for x, _ in order[r]]
            cnt = [sum(1 for _, ro in order[r] if ro == q) for q in range(4)]
            print(f"    rank {r}: {np.median(xs):7.0f}  roles {cnt}")
        span = [np.max(t[d, b, :, nph, 1]) - np.min(t[d, b, :, 0, 0]) for b in blocks]
        print(f"  loop span median {np.median(span):.0f} cycles")
    eng.close()


if __name__ == "__main__":
    main()
