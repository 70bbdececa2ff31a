#!/bin/bash
# Interleaved A/B of two library builds on the 500k one-GPU headline (bench.py, reduced legs):
# bash tools/head_ab.sh OUT LIB_A LIB_B [reps]
set -e -o pipefail
O=gpurun_out/$1; A=$2; B=$3; R=${4:-3}
mkdir -p $O
BB="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --no-provider --steps 20 --warmup 5"
for rep in $(seq 1 $R); do
  for lib in $A $B; do
    n=$(basename $lib .so)
    BBX=$BB
    FREI_HIP_LIB=$lib timeout -k 10 200 $BBX > $O/${n}_$rep.json 2>/dev/null
    python3 -c "
import json; d=json.load(open('$O/${n}_$rep.json')); r=d['rad_eq']
print('$n rep $rep', round(d['ms_per_step']*1e3,2), 'us/iter', '%.4g' % d['value'], 'sweep', round(d['roofline']['avg_launch_ms']*1e3,2), 'us; rad_eq warm', round(r['iters_per_s']), 'it/s, incl setup', round(r['iters_per_s_incl_setup']), r.get('incl_setup', {}).get('full_k3', {}).get('iters_per_s'))"
  done
done
