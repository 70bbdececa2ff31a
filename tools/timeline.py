"""Per-sweep timeline of the T-P loop from a rocprofv3 kernel trace.

    python tools/timeline.py path/to/run_kernel_trace.csv [SWEEP_GRID_X]

SWEEP_GRID_X keeps only the sweeps of that grid size (e.g. 500224 for the 500k one-lane sweep,
leaving out the batched and per-atmosphere legs of a full bench run).

For every sweep -> reduce -> (all-gather) -> update cycle (or sweep -> fused update) it attributes the kernel durations
and the idle gaps between consecutive kernels (end of one to start of the next), then
prints the medians: what a T-P half-iteration costs beyond the sweep itself.
"""
import csv
import statistics
import sys


def kind(name):
    for k in ("sweep", "reduce_kernel", "update_kernel", "update_fused", "ncclDevKernel",
              "AllGather"):
        if k in name:
            return {"reduce_kernel": "reduce", "update_kernel": "update",
                    "update_fused": "update",
                    "ncclDevKernel": "allgather", "AllGather": "allgather"}.get(k, k)
    return None


def main(path, grid=None):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            k = kind(r["Kernel_Name"])
            if k == "sweep" and grid is not None and r["Grid_Size_X"] != grid:
                k = None
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k,
                         r["Kernel_Name"][:60]))
    rows.sort()
    cycles = []
    cur = None
    prev_end = None
    for s, e, k, name in rows:
        if k == "sweep":
            if cur is not None and "update" in cur:
                cycles.append(cur)
            cur = {"sweep": (e - s) / 1e3, "gap_in": None if prev_end is None else (s - prev_end) / 1e3}
        elif cur is not None and k in ("reduce", "update", "allgather"):
            cur[k] = (e - s) / 1e3
            cur["gap_" + k] = (s - prev_end) / 1e3
        elif cur is not None and k is None:
            cur = None          # another kernel interleaved: not a clean cycle
        prev_end = e
    if not cycles:
        print("no sweep/reduce/update cycles found")
        return
    keys = ["sweep", "gap_reduce", "reduce", "gap_allgather", "allgather", "gap_update",
            "update", "gap_in"]
    print(f"{len(cycles)} cycles (median microseconds):")
    tot = 0.0
    for k in keys:
        v = [c[k] for c in cycles if c.get(k) is not None]
        if v:
            m = statistics.median(v)
            tot += m
            print(f"  {k:>14s} {m:9.2f}")
    print(f"  {'half-iteration':>14s} {tot:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
