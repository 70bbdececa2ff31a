#!/bin/bash
# Issue-priority modes of the 500k sweep (two wavelengths per lane), interleaved on one box:
# progress quartiles (1, default), rotating by trip and block (2), none (0).
set -o pipefail
O=gpurun_out/${1:-r04prio}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  for t in prio1 prio4; do
    FREI_HIP_LIB=ablib/$t.so timeout -k 10 120 python3 bench.py $B > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_$rep.json')); print('$t', $rep, '500k %.4f ms sweep %.2f us' % (a['ms_per_step'], a['roofline']['avg_launch_ms']*1e3), flush=True)" | tee -a $O/summary.txt
  done
done
