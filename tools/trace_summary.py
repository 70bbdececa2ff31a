"""Per-kernel summary of a rocprofv3 --kernel-trace CSV that separates real sweep launches
from the no-op launches the device-resident T-P loop issues after convergence (kernels
that see the convergence flag return immediately; the host polls one chunk behind).

    python tools/trace_summary.py run_kernel_trace.csv [bench.json]
"""
import csv
import json
import statistics as st
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = {}
    for r in rows:
        by.setdefault(r["Kernel_Name"], []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':70s} {'calls':>6s} {'mean_us':>10s} {'median_us':>10s} {'no-op':>6s} {'mean_real_us':>12s}")
    for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        med = st.median(d)
        real = [x for x in d if x > 0.05 * med]
        print(f"{name[:70]:70s} {len(d):6d} {st.mean(d):10.2f} {med:10.2f} "
              f"{len(d) - len(real):6d} {st.mean(real):12.2f}")
    if len(sys.argv) > 2:
        b = json.load(open(sys.argv[2]))
        print(f"\nbench.py HIP-event average of the sweep kernel: "
              f"{b['roofline']['avg_launch_ms'] * 1e3:.2f} us over {b['roofline']['launches']} launches")


if __name__ == "__main__":
    main()
