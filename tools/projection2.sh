#!/bin/bash
# Projection with cost-balanced slices: every even slice r/N of the 500k grid (bench --lam-slice,
# one-rank P2P) gives its sweep time; balanced_edges re-splits; every balanced slice is measured
# again.  The N-GPU step is the slowest rank's; the one-GPU 500k step on the same box.
set -e -o pipefail
O=gpurun_out/${1:-proj2}
mkdir -p $O
B="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --steps 40 --warmup 5"
for r in 1 2; do
  timeout -k 10 200 $B > $O/bench500_$r.json 2>/dev/null
  python3 -c "import json; d=json.load(open('$O/bench500_$r.json')); print('500k one GPU', round(d['ms_per_step']*1e3,2), 'us per T-P iteration')"
done
for n in 8 4 2; do
  python3 - $n $O <<'PY'
import json, subprocess, sys
n, O = int(sys.argv[1]), sys.argv[2]
sys.path.insert(0, ".")
from frei_amd.engine import partition, balanced_edges
B = ["python3", "bench.py", "--no-binning", "--no-cpu-baseline", "--no-c5", "--no-per-species",
     "--no-chemistry", "--rad-eq-max", "1", "--steps", "40", "--warmup", "5", "--force-comm"]
def run(lo, hi, tag):
    out = subprocess.run(["timeout", "-k", "10", "150"] + B + ["--lam-slice", f"{lo}:{hi}"],
                         capture_output=True, text=True, check=True).stdout
    d = json.loads(out)
    open(f"{O}/{tag}_{lo}_{hi}.json", "w").write(out)
    return d["ms_per_step"] * 1e3, d["roofline"]["avg_launch_ms"]
even = [partition(500000, n, r)[0] for r in range(n)] + [500000]
res = [run(a, b, f"even{n}") for a, b in zip(even, even[1:])]
edges = balanced_edges(even, [s for _, s in res])
bal = [run(a, b, f"bal{n}") for a, b in zip(edges, edges[1:])]
print(f"N={n} even: max {max(t for t, _ in res):.2f} us ({' '.join(f'{t:.1f}' for t, _ in res)})")
print(f"N={n} balanced edges {edges}: max {max(t for t, _ in bal):.2f} us ({' '.join(f'{t:.1f}' for t, _ in bal)})")
PY
done
