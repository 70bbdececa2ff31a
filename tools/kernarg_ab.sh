#!/bin/bash
set -o pipefail
O=gpurun_out/karg
mkdir -p $O
B="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --no-provider --rad-eq-max 1 --steps 40 --warmup 5 --force-comm --lam-slice 312500:375000"
for rep in 1 2; do
  for v in def 1 0; do
    if [ $v = def ]; then E=""; else E="HIP_FORCE_DEV_KERNARG=$v"; fi
    env $E timeout -k 10 150 $B > $O/k${v}_$rep.json 2> $O/k${v}_$rep.err || { echo failed; exit 1; }
    python3 -c "import json; d=json.load(open('$O/k${v}_$rep.json')); print('kernarg $v rep $rep', round(d['ms_per_step']*1e3,2), 'us per T-P iteration')"
  done
done
