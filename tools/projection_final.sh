#!/bin/bash
# Final-tree projection at N = 8: the one-GPU 500k step, then every even slice r/8 of the 500k
# grid as one rank (bench --lam-slice, one-rank P2P).  The N-GPU step is the slowest rank's.
set -e -o pipefail
O=gpurun_out/${1:-projf}
mkdir -p $O
B="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --steps 40 --warmup 5"
timeout -k 10 200 $B > $O/bench500.json 2>/dev/null
python3 -c "import json; d=json.load(open('$O/bench500.json')); print('500k one GPU', round(d['ms_per_step']*1e3,2), 'us per T-P iteration')"
for r in 0 1 2 3 4 5 6 7; do
  lo=$((r * 62500)); hi=$(((r + 1) * 62500))
  timeout -k 10 150 $B --force-comm --lam-slice $lo:$hi > $O/slice_$r.json 2>/dev/null
  python3 -c "import json; d=json.load(open('$O/slice_$r.json')); print('slice $r/8', round(d['ms_per_step']*1e3,2), 'us per T-P iteration, sweep', round(d['roofline']['avg_launch_ms']*1e3,2), 'us')"
done
