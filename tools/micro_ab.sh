#!/bin/bash
# Micro A/Bs, alternating on one box: 1/chi with one Newton step (abv/rcp1.so) at 500k and at the
# 8-GPU slice; the producer/consumer consumer at priority 3 (abv/prio3.so) at the slice.
set -e -o pipefail
O=gpurun_out/${1:-micro}
mkdir -p $O
B="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1"
for r in 1 2 3; do
  for lib in default rcp1 prio3; do
    if [ $lib = default ]; then unset FREI_HIP_LIB; else export FREI_HIP_LIB=abv/$lib.so; fi
    timeout -k 10 120 $B --steps 20 > $O/b500_${lib}_$r.json 2>/dev/null
    timeout -k 10 120 $B --n-lam 62500 --steps 40 --warmup 5 --force-comm > $O/b62_${lib}_$r.json 2>/dev/null
    python3 -c "import json; f=lambda n: json.load(open('$O/'+n+'_${lib}_$r.json')); print('$lib', $r, '500k', round(f('b500')['ms_per_step']*1e3,1), 'sweep', round(f('b500')['roofline']['avg_launch_ms']*1e3,1), '62.5k p2p', round(f('b62')['ms_per_step']*1e3,2))"
  done
done
unset FREI_HIP_LIB
