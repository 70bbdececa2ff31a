#!/bin/bash
# Where the producer/consumer sweep's loop time goes at the 8-GPU slice size (62.5k lambda):
# default, producers with trivial coefficients (abv/noprod.so), consumers that only meet the
# barriers (abv/nocons.so), producers loading two phases ahead (FREI_PIPE_PF=2).  Ablation
# builds give wrong results: timing only.
set -e -o pipefail
O=gpurun_out/${1:-ablate}
mkdir -p $O
B="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --n-lam 62500 --steps 40 --warmup 5 --force-comm"
for r in 1 2; do
  for v in ${VARIANTS:-default noprod nocons pf2}; do
    unset FREI_HIP_LIB FREI_PIPE_PF
    case $v in noprod|nocons|nored|nostore|stalehot|spf2|ring0) export FREI_HIP_LIB=abv/$v.so;; pf2) export FREI_PIPE_PF=2;; esac
    timeout -k 10 120 $B > $O/b62_${v}_$r.json 2>$O/b62_${v}_$r.err
    python3 -c "import json; d=json.load(open('$O/b62_${v}_$r.json')); print('$v', $r, '62.5k p2p', round(d['ms_per_step']*1e3,2), 'sweep', round(d['roofline']['avg_launch_ms']*1e3,2), d.get('sweep_path',{}).get('pipe'))"
  done
done
