#!/bin/bash
# Multi-GPU projection on one MI355X: every rank's slice r/N of the 500k grid (N = 2, 4, 8) with the
# one-rank P2P exchange (production build, chained launches as the default), and the one-GPU
# bench at 500k on the same box (3 runs).  The N-GPU step is the slowest rank's.
set -e -o pipefail
O=gpurun_out/${1:-proj}
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --steps 40 > $O/bench500_$r.json 2>/dev/null
  python3 -c "import json; d=json.load(open('$O/bench500_$r.json')); print('500k one GPU', round(d['ms_per_step']*1e3,2), 'us per T-P iteration; sweep', round(d['roofline']['avg_launch_ms']*1e3,2))"
done
T="timeout -k 10 120 python3 tools/trace_probe.py --n-lam 500000 --iters 40 --p2p"
for n in 8 4 2; do
  for r in $(seq 0 $((n-1))); do
    $T --slice $r/$n 2>/dev/null | tee -a $O/slices_$n.txt
  done
done
