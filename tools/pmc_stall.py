"""Per-wave stall fractions and instruction mix of the sweep kernels from rocprofv3 SQ passes.

    python tools/pmc_stall.py DIR [DIR ...] [--n-lam N --n-layers L]

Each DIR holds one rocprofv3 --pmc pass (run_counter_collection.csv).  For every sweep kernel
name: the median over its dispatches of each counter; SQ_WAIT_ANY / SQ_WAIT_INST_ANY /
SQ_ACTIVE_INST_* as fractions of SQ_WAVE_CYCLES, SQ_INSTS_* per 64 flux updates, and
valu_busy = 4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8).
"""
import csv
import statistics
import sys


def main():
    dirs = [a for a in sys.argv[1:] if not a.startswith("--")]
    opts = dict(a.lstrip("-").split("=") for a in sys.argv[1:] if a.startswith("--"))
    upd = (int(opts.get("n-layers", 60)) - 1) * int(opts.get("n-lam", 500000))
    per = {}
    for d in dirs:
        for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
            name = r["Kernel_Name"]
            if "sweep" not in name:
                continue
            short = name.split("(")[0].replace("void frei::", "")
            per.setdefault(short, {}).setdefault(r["Counter_Name"], {}).setdefault(
                (d, r["Dispatch_Id"]), 0.0)
            per[short][r["Counter_Name"]][(d, r["Dispatch_Id"])] += float(r["Counter_Value"])
    for k, cs in per.items():
        med = {c: statistics.median(v.values()) for c, v in cs.items()}
        wc = med.get("SQ_WAVE_CYCLES")
        out = [k]
        for c, v in sorted(med.items()):
            if c.startswith(("SQ_WAIT", "SQ_ACTIVE")) and wc:
                out.append(f"{c[3:]} {v / wc:.3f}")
            elif c.startswith("SQ_INSTS"):
                out.append(f"{c[3:]}/64upd {v * 64 / upd:.1f}")
        if "SQ_ACTIVE_INST_VALU" in med and "GRBM_GUI_ACTIVE" in med:
            out.append(f"valu_busy {4 * med['SQ_ACTIVE_INST_VALU'] / (1024 * med['GRBM_GUI_ACTIVE'] / 8):.3f}")
        print("  ".join(out))


if __name__ == "__main__":
    main()
