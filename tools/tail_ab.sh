#!/bin/bash
# Trailing update A/B at the 8-GPU slice (as one rank of N = 8 runs it: slice 5 of the 500k grid,
# with the one-rank P2P exchange and without), FREI_TAIL=1 / 0 interleaved, then the 500k step.
set -e -o pipefail
O=gpurun_out/${1:-tail_ab}
mkdir -p $O
B="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --no-provider --rad-eq-max 1 --steps 40 --warmup 5"
for rep in 1 2; do
  for comm in p2p local; do
    F=""; [ $comm = p2p ] && F="--force-comm"
    for t in 1 0; do
      FREI_TAIL=$t timeout -k 10 150 $B $F --lam-slice 312500:375000 > $O/s5_${comm}_tail${t}_$rep.json 2>/dev/null
      python3 -c "import json; d=json.load(open('$O/s5_${comm}_tail${t}_$rep.json')); print('slice 5/8 $comm tail $t rep $rep', round(d['ms_per_step']*1e3,2), 'us per T-P iteration, sweep', round(d['roofline']['avg_launch_ms']*1e3,2), 'us, tail', d['sweep_path'].get('tail'))"
    done
  done
done
if [ -z "$NO500" ]; then
timeout -k 10 200 $B > $O/bench500.json 2>/dev/null
python3 -c "import json; d=json.load(open('$O/bench500.json')); print('500k one GPU', round(d['ms_per_step']*1e3,2), 'us per T-P iteration')"
fi
