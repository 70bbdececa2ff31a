#!/bin/bash
# The 2- and 4-GPU slices (250k, 125k lambda, one-rank P2P exchange): the automatic sweep form
# against two wavelengths per lane forced and the grouped-lane Q = 2 form, one box.
set -o pipefail
O=gpurun_out/${1:-r04sizes}
mkdir -p $O
for sl in 0:250000 0:125000; do
  B="--no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --steps 30 --warmup 5 --force-comm --lam-slice $sl"
  for rep in 1 2; do
    for t in auto lam2 q2 one; do
      case $t in
        auto) E="FREI_X=0";;
        lam2) E="FREI_LAM2=1 FREI_SHARED=0 FREI_GROUP_Q=1 FREI_PIPE=0";;
        q2) E="FREI_GROUP_Q=2 FREI_PIPE=0";;
        one) E="FREI_LAM2=0 FREI_SHARED=0 FREI_GROUP_Q=1 FREI_PIPE=0";;
      esac
      env $E timeout -k 10 120 python3 bench.py $B > $O/${t}_${sl/:/_}_$rep.json 2> /dev/null || { echo "bench $t $sl failed"; exit 3; }
      python3 -c "import json; a=json.load(open('$O/${t}_${sl/:/_}_$rep.json')); p=a['sweep_path']; print('$sl', '$t', $rep, '%.2f us per T-P iteration, sweep %.2f us' % (a['ms_per_step']*1e3, a['roofline']['avg_launch_ms']*1e3), 'lam2', p.get('lam2'), 'paired', p['paired'], 'quad', p['quad'], 'pipe', p['pipe'], 'lds', p['lds_steps'], flush=True)" | tee -a $O/summary.txt
    done
  done
done
