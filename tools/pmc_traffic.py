"""Summarise rocprofv3 PMC runs into per-launch HBM traffic of the sweep kernel.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [--n-lam N --n-layers L --species S]
                                [--kernel NAME --contracted 0|1]

--kernel (default sweep_pair_kernel, the headline sweep) selects the dispatches by name: a bench
run also holds the per-species leg's sweep (sweep_fast_kernel, --contracted=0).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts exactly half
of the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM section), so
HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE.  Median over the sweep-kernel dispatches of each
kernel (the timed T-P steps; excludes the rad-eq run's one full-write final emit).
"""
import statistics
import csv
import json
import sys


def per_kernel(path, counter, name):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or name not in r["Kernel_Name"]:
            continue
        vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]) * 1024.0)
    return {k: statistics.median(v) for k, v in vals.items()}


def main():
    fdir, wdir, out = sys.argv[1:4]
    opts = dict(a.lstrip("-").split("=") for a in sys.argv[4:])
    n_lam = int(opts.get("n-lam", 500000))
    nL = int(opts.get("n-layers", 60))
    S = int(opts.get("species", 8))
    contracted = opts.get("contracted", "1") == "1"   # K3: the sweep reads one table
    name = opts.get("kernel", "sweep_pair_kernel")
    fetch = per_kernel(f"{fdir}/run_counter_collection.csv", "FETCH_SIZE", name)
    write = per_kernel(f"{wdir}/run_counter_collection.csv", "WRITE_SIZE", name)
    kernels = {}
    for k in fetch:
        rd = 2.0 * fetch[k]
        wr = write.get(k, 0.0)
        kernels[k] = {"fetch_size_B": fetch[k], "read_B_corrected": rd, "write_B": wr,
                      "hbm_B": rd + wr}
    mean = sum(v["hbm_B"] for v in kernels.values()) / max(len(kernels), 1)
    S_run = 1 if contracted else S
    alg = (8 + 8 + 16 * S_run) * (nL - 1) * n_lam   # T-P loop sweep (dead stores removed)
    json.dump({"workload": {"n_lam": n_lam, "n_layers": nL, "species": S,
                            "contracted": contracted},
               "kernels": kernels, "hbm_B_per_launch": mean,
               "algorithmic_B_per_launch": alg, "traffic_over_algorithmic": mean / alg,
               "correction": "HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving)"},
              open(out, "w"), indent=1)
    print(json.dumps({"hbm_B_per_launch": mean, "ratio": mean / alg}))


if __name__ == "__main__":
    main()
