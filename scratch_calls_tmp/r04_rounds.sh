#!/bin/bash
# Sweep time per lambda vs how many rounds of blocks the grid needs: 1280 resident blocks at
# 5 waves per SIMD (256 CUs x 5), so 327,680 lambda = 1 round, 500k = 1.53, 655,360 = 2.
set -o pipefail
O=gpurun_out/${1:-r04rounds}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5 --rad-eq-max 1"
for rep in 1 2; do
  for n in 327680 409600 500224 655360; do
    timeout -k 10 120 python3 bench.py $B --n-lam $n > $O/n${n}_$rep.json 2> /dev/null || { echo "bench $n failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/n${n}_$rep.json')); s=a['roofline']['avg_launch_ms']*1e3; print('n $n rep $rep sweep %.2f us = %.3f ns per lambda; iteration %.1f us' % (s, s*1e3/$n, a['ms_per_step']*1e3), flush=True)" | tee -a $O/summary.txt
  done
done
