#!/bin/bash
# Is the slow long-wavelength slice a property of its wavelengths or of the temperatures its
# one-rank run drifts to?  Slices 0/8 and 7/8 timed right after the initial T (warm-up 0, 4
# steps) and after 40 iterations (warm-up 40, 20 steps); and each slice's T after the warm-up.
set -e -o pipefail
O=gpurun_out/${1:-tdep}
mkdir -p $O
B="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --force-comm"
for r in 0 7; do
  lo=$((r*62500)); hi=$(((r+1)*62500))
  for wu in 0 40; do
    timeout -k 10 120 $B --lam-slice $lo:$hi --warmup $wu --steps 20 > $O/s${r}_w$wu.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/s${r}_w$wu.json')); print('slice $r warmup $wu', round(d['ms_per_step']*1e3,1), 'us; sweep', round(d['roofline']['avg_launch_ms']*1e3,2))"
  done
done
timeout -k 10 300 python3 tools/slice_globalT.py --n 8 --iters 40 > $O/globalT.txt 2>&1; cat $O/globalT.txt
