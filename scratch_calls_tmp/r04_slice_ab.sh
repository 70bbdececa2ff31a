#!/bin/bash
# The 8-GPU slice (62.5k lambda, one-rank P2P exchange): sweep forms interleaved on one box,
# after the round-4 register savings (exp-form Planck) changed every form's occupancy.
set -o pipefail
O=gpurun_out/${1:-r04slice}
mkdir -p $O
B="--no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --steps 40 --warmup 5 --force-comm --lam-slice 0:62500"
for rep in 1 2; do
  for t in auto pipe0 q2 q4 q2w8 q4w8 q1; do
    case $t in
      auto) E="FREI_X=0";;
      pipe0) E="FREI_PIPE=0";;
      q2) E="FREI_PIPE=0 FREI_GROUP_Q=2";;
      q4) E="FREI_PIPE=0 FREI_GROUP_Q=4";;
      q2w8) E="FREI_PIPE=0 FREI_GROUP_Q=2 FREI_GROUP_WAVES=8";;
      q4w8) E="FREI_PIPE=0 FREI_GROUP_Q=4 FREI_GROUP_WAVES=8";;
      q1) E="FREI_PIPE=0 FREI_GROUP_Q=1";;
    esac
    env $E timeout -k 10 120 python3 bench.py $B > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_$rep.json')); print('$t', $rep, 'slice0 %.2f us per T-P iteration, sweep %.2f us, path %s' % (a['ms_per_step']*1e3, a['roofline']['avg_launch_ms']*1e3, a['sweep_path']), flush=True)" | tee -a $O/summary.txt
  done
done
