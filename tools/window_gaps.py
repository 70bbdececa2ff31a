"""The bench's timed window, read off a rocprofv3 kernel trace of `bench.py`.

    python tools/window_gaps.py run_kernel_trace.csv [--warmup 3] [--steps 20]

bench.py's headline is the first T-P loop after the engine's setup: `warmup` untimed
iterations, then `steps` timed ones (2 sweeps + 2 fused updates each).  This takes, in launch
order, the kernels from the first 500k-grid sweep on, skips the warm-up iterations and reports
for the timed ones: the sum of sweep and update durations, the idle gaps between consecutive
kernels, the window's span (first timed sweep's start to last update's end), and the sweep
durations in order (the clock management shows there as a drift within the window).
"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--grid", default=None, help="sweep Grid_Size_X (default: the first sweep's)")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r["Grid_Size_X"]))
    rows.sort()
    first = next(i for i, r in enumerate(rows)
                 if "sweep" in r[2] and (a.grid is None or r[3] == a.grid))
    grid = a.grid or rows[first][3]
    seq = []
    for r in rows[first:]:
        if "sweep" in r[2] and r[3] == grid:
            seq.append(("sweep", r))
        elif "update" in r[2] or "reduce" in r[2]:
            seq.append(("update", r))
        else:
            break
        if sum(1 for k, _ in seq if k == "sweep") > 2 * (a.warmup + a.steps):
            seq.pop()
            break
    n_sw = 0
    start = None
    for i, (k, _) in enumerate(seq):
        if k == "sweep":
            if n_sw == 2 * a.warmup:
                start = i
                break
            n_sw += 1
    win = seq[start:]
    sweeps = [(e - s) / 1e3 for k, (s, e, _, _) in win if k == "sweep"]
    upds = [(e - s) / 1e3 for k, (s, e, _, _) in win if k == "update"]
    gaps = [(win[i][1][0] - win[i - 1][1][1]) / 1e3 for i in range(1, len(win))]
    span = (win[-1][1][1] - win[0][1][0]) / 1e3
    it = len(sweeps) / 2
    print(f"timed window: {len(sweeps)} sweeps, {len(upds)} updates over {it:.0f} T-P iterations "
          f"(grid {grid}); span {span:.1f} us = {span / it:.2f} us per iteration")
    print(f"  per iteration: sweeps {sum(sweeps) / it:.2f} us, updates {sum(upds) / it:.2f} us, "
          f"gaps {sum(gaps) / it:.2f} us")
    print(f"  sweep us: median {statistics.median(sweeps):.2f}, min {min(sweeps):.2f}, "
          f"max {max(sweeps):.2f}; update median {statistics.median(upds):.2f}; gap median "
          f"{statistics.median(gaps):.2f}, max {max(gaps):.2f}")
    print("  sweep durations in order:", " ".join(f"{x:.0f}" for x in sweeps))


if __name__ == "__main__":
    main()
