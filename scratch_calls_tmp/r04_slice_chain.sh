#!/bin/bash
# The 8-GPU slice: producer/consumer sweep unchained (auto) vs chained (FREI_CHAIN=2), one box.
set -o pipefail
O=gpurun_out/${1:-r04slch}
mkdir -p $O
B="--no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --steps 40 --warmup 5 --force-comm --lam-slice 0:62500"
for rep in 1 2 3; do
  for t in auto chain2; do
    if [ $t = auto ]; then E="FREI_X=0"; else E="FREI_CHAIN=2"; fi
    env $E timeout -k 10 120 python3 bench.py $B > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_$rep.json')); print('$t', $rep, 'slice0 %.2f us per T-P iteration' % (a['ms_per_step']*1e3), flush=True)" | tee -a $O/summary.txt
  done
done
