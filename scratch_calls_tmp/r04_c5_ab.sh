#!/bin/bash
# C5 batched leg (32 atmospheres x 100k lambda): default sweep form vs two wavelengths per lane
# (FREI_LAM2=1 FREI_SHARED=0), one box, interleaved.
set -o pipefail
O=gpurun_out/${1:-r04c5}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-chemistry --no-per-species --steps 5 --warmup 2 --rad-eq-max 1"
for rep in 1 2 3; do
  for t in auto lam2; do
    if [ $t = auto ]; then E="FREI_X=0"; else E="FREI_LAM2=1 FREI_SHARED=0"; fi
    env $E timeout -k 10 300 python3 bench.py $B > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_$rep.json'))['c5_batched']; print('$t', $rep, 'C5 %.4e updates/s, %.3f ms per step, rad-eq %.3f s' % (a['updates_per_s'], a['ms_per_step'], a['rad_eq']['wall_s']), flush=True)" | tee -a $O/summary.txt
  done
done
