#!/bin/bash
# K6 binning: nontemporal table stores (nt) vs plain stores (base), interleaved, one box.
set -o pipefail
O=gpurun_out/${1:-r04binnt}
mkdir -p $O
B="--no-cpu-baseline --no-c5 --no-chemistry --no-per-species --steps 2 --warmup 1 --rad-eq-max 1"
for rep in 1 2 3; do
  for t in nt base; do
    FREI_HIP_LIB=ablib/$t.so timeout -k 10 300 python3 bench.py $B > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; b=json.load(open('$O/${t}_$rep.json'))['k6_binning']; print('$t', $rep, 'groupies %.3f ms frac %.3f, exact %.3f ms frac %.3f' % (b['groupies']['avg_launch_ms'], b['groupies']['roofline']['frac'], b['exact']['avg_launch_ms'], b['exact']['roofline']['frac']), flush=True)" | tee -a $O/summary.txt
  done
done
