"""K7 (batched contraction) timing of one library build: the C5 workload of bench.py's c5 leg
(32 atmospheres x 60 x 100k x 8 species), contraction kernel HIP-event ms and GB/s, `reps`
fresh contexts.  FREI_HIP_LIB selects the build.   python tools/k7_ab.py [reps]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from frei_amd.batch import BatchEngine
    from frei_amd.opacity import SeparableTable
    from frei_amd.tp import temperature_grid
    from frei_amd.workloads import c3
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    w = c3(n_lam=100_000)
    T_refs = np.arange(1000.0, 2401.0, 200.0)
    loggs = np.array([2.5, 3.0, 3.5, 4.0])
    T0 = np.array([temperature_grid(w["p"], t, 0.1, 0.1) for t in T_refs for _ in loggs])
    g = np.array([10.0 ** lg for _ in T_refs for lg in loggs])
    T_nodes = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 16)
    fT = (T_nodes / 1000.0) ** 0.5
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], fT, w["p"], T_nodes)
            for s, n in enumerate(w["names"])}
    mmr = np.broadcast_to(w["mmr"], (len(g),) + w["mmr"].shape)
    out = []
    for _ in range(reps):
        eng = BatchEngine(w["lam"], w["p"], tabs, g=g, mmr=mmr)
        try:
            eng.state_init(T0)
            eng.synchronize()
            k = eng.contract_timing()
            out.append(dict(ms=k["ms"], GBps=k["bytes"] / k["ms"] / 1e6,
                            zero_ms=eng.setup_timing()["eff_zero"]))
            # the same contraction again into the now-touched buffer (metadata rebuilt)
            eng.set_option("rec_sweep", -1)
            eng.state_init(T0)
            eng.synchronize()
            k = eng.contract_timing()
            out.append(dict(again_ms=k["ms"], GBps=k["bytes"] / k["ms"] / 1e6))
        finally:
            eng.close()
    print(json.dumps({"lib": os.environ.get("FREI_HIP_LIB", "default"),
                      "k7_mfma": os.environ.get("FREI_K7_MFMA", "1"), "runs": out}))


if __name__ == "__main__":
    main()
