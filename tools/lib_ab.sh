#!/bin/bash
# Interleaved A/B of two library builds at the 8-GPU slice (slice 5/8 of the 500k grid, one-rank
# P2P): bash tools/lib_ab.sh OUT LIB_A LIB_B [reps]
set -e -o pipefail
O=gpurun_out/$1; A=$2; B=$3; R=${4:-3}
mkdir -p $O
BB="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --no-provider --rad-eq-max 1 --steps 40 --warmup 5 --force-comm --lam-slice 312500:375000"
for rep in $(seq 1 $R); do
  for lib in $A $B; do
    n=$(basename $lib .so)
    FREI_HIP_LIB=$lib timeout -k 10 150 $BB > $O/${n}_$rep.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/${n}_$rep.json')); print('$n rep $rep', round(d['ms_per_step']*1e3,2), 'us per T-P iteration, sweep', round(d['roofline']['avg_launch_ms']*1e3,2), 'us')"
  done
done
