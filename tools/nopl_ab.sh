#!/bin/bash
# A/B: the producer/consumer sweep without its repeated Planck value per producer and phase
# (abv/nopl.so, -DFREI_PIPE_NOPL: results wrong, timing only) at the 8-GPU slice size.
set -e -o pipefail
O=gpurun_out/${1:-nopl}
mkdir -p $O
B="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1"
for r in 1 2 3; do
  for lib in default nopl; do
    if [ $lib = default ]; then unset FREI_HIP_LIB; else export FREI_HIP_LIB=abv/$lib.so; fi
    timeout -k 10 120 $B --n-lam 62500 --steps 40 --warmup 5 --force-comm > $O/b62_${lib}_$r.json 2>/dev/null
    python3 -c "import json; f=lambda n: json.load(open('$O/'+n+'_${lib}_$r.json')); d=f('b62'); print('$lib', $r, '62.5k p2p', round(d['ms_per_step']*1e3,2), 'sweep', round(d['roofline']['avg_launch_ms']*1e3,2), d.get('sweep_path',{}).get('pipe'))"
  done
done
