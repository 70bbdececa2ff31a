"""Per-kernel summary of a rocprofv3 --kernel-trace CSV that separates real sweep launches
from the no-op launches the device-resident T-P loop issues after convergence (kernels
that see the convergence flag return immediately; the host polls one chunk behind).

    python tools/trace_summary.py run_kernel_trace.csv|rocprof_dir|run_results.db [bench.json]

rocprofv3 7.x writes an SQLite database by default (no --output-format csv); both are read.
"""
import glob
import os
import sqlite3
import csv
import json
import statistics as st
import sys


def load(path):
    """Kernel dispatches as dicts with Kernel_Name / Start_Timestamp / End_Timestamp (ns)."""
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) or \
            glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        path = cands[0]
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        rows = [dict(Kernel_Name=n, Start_Timestamp=a, End_Timestamp=b)
                for n, a, b in con.execute("select name, start, end from kernels")]
    else:
        rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def main():
    rows = load(sys.argv[1])
    by = {}
    for r in rows:
        # launches of one kernel with different grids (e.g. the 500k-lambda headline sweep and
        # the batched C5 sweep) are separate rows
        grid = ""
        if "Grid_Size_X" in r:
            grid = f"{int(r['Grid_Size_X']) // max(int(r.get('Workgroup_Size_X', 1)), 1)}"
            if int(r.get("Grid_Size_Y", 1)) > 1:
                grid += f"x{r['Grid_Size_Y']}"
        by.setdefault((r["Kernel_Name"], grid), []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':62s} {'grid':>9s} {'calls':>6s} {'mean_us':>10s} {'median_us':>10s} "
          f"{'no-op':>6s} {'mean_real_us':>12s}")
    for (name, grid), d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        med = st.median(d)
        real = [x for x in d if x > 0.05 * med]
        print(f"{name[:62]:62s} {grid:>9s} {len(d):6d} {st.mean(d):10.2f} {med:10.2f} "
              f"{len(d) - len(real):6d} {st.mean(real):12.2f}")
    if len(sys.argv) > 2:
        b = json.load(open(sys.argv[2]))
        print(f"\nbench.py HIP-event average of the sweep kernel: "
              f"{b['roofline']['avg_launch_ms'] * 1e3:.2f} us over {b['roofline']['launches']} launches")


if __name__ == "__main__":
    main()
