#!/bin/bash
# Per-species sweep (8 tables, no K3): one coefficient block of two steps (default, 148 VGPRs,
# 3 waves per SIMD) vs one step (FREI_PREFETCH_DEPTH=1: 97 VGPRs, 5 waves per SIMD), one box.
set -o pipefail
O=gpurun_out/${1:-r04ps}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --steps 4 --warmup 2 --rad-eq-max 1"
for rep in 1 2 3; do
  for t in d2 d1; do
    if [ $t = d2 ]; then E="FREI_X=0"; else E="FREI_PREFETCH_DEPTH=1"; fi
    env $E timeout -k 10 200 python3 bench.py $B > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_$rep.json'))['per_species']; print('$t', $rep, 'per-species %.4f ms per T-P iteration, sweep %.1f us, frac %.3f' % (a['ms_per_step'], a['roofline']['avg_launch_ms']*1e3, a['roofline']['frac']), flush=True)" | tee -a $O/summary.txt
  done
done
