"""VALU utilisation of the sweep kernel from a rocprofv3 SQ counter pass.

    python tools/pmc_valu.py SQ_DIR OUT.json [--n-lam N --n-layers L --kernel NAME]

Counters (one pass): SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_WAVES, SQ_WAVE_CYCLES,
SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE.  SQ_ACTIVE_INST_VALU counts quad-cycles summed over waves;
GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md), so
  valu_busy = 4 * SQ_ACTIVE_INST_VALU / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
and VALU wave-instructions per flux update = SQ_INSTS_VALU * 64 / updates per launch.
Median over the dispatches of the kernel named by --kernel (default sweep_pair_kernel, the
headline sweep; sweep_fast_kernel for the per-species leg).
"""
import csv
import json
import statistics
import sys


def main():
    d, out = sys.argv[1:3]
    opts = dict(a.lstrip("-").split("=") for a in sys.argv[3:])
    n_lam = int(opts.get("n-lam", 500000))
    nL = int(opts.get("n-layers", 60))
    name = opts.get("kernel", "sweep_pair_kernel")
    per = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if name not in r["Kernel_Name"]:
            continue
        key = (r["Dispatch_Id"], r["Kernel_Name"])
        per.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    rows = [v for v in per.values() if "SQ_INSTS_VALU" in v and "GRBM_GUI_ACTIVE" in v]
    med = {k: statistics.median(r[k] for r in rows) for k in rows[0]}
    updates = (nL - 1) * n_lam
    busy = 4 * med["SQ_ACTIVE_INST_VALU"] / (1024 * med["GRBM_GUI_ACTIVE"] / 8)
    res = {"dispatches": len(rows), "median_counters": med,
           "valu_busy": busy,
           "valu_insts_per_update": med["SQ_INSTS_VALU"] * 64 / updates,
           "waves": med.get("SQ_WAVES"),
           "formula": "valu_busy = 4*SQ_ACTIVE_INST_VALU / (1024 * GRBM_GUI_ACTIVE/8)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({"valu_busy": busy, "valu_insts_per_update": res["valu_insts_per_update"]}))


if __name__ == "__main__":
    main()
