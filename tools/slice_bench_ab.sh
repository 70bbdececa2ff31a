#!/bin/bash
# bench.py at the 8-GPU slice (62.5k) with the one-rank P2P exchange forced on, alternating
# sweep forms: default (producer/consumer), producer/consumer with records formed in the sweep,
# and two lanes per wavelength (FREI_PIPE=0 -> grouped-lane Q = 2).
set -e -o pipefail
O=${1:-gpurun_out/slice}
mkdir -p $O
B="python3 bench.py --n-lam 62500 --steps 40 --warmup 5 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --force-comm"
for r in 1 2 3; do
  for v in default pipe_rec q2; do
    case $v in
      default) env="" ;;
      pipe_rec) env="FREI_REC_SWEEP=1" ;;
      q2) env="FREI_PIPE=0" ;;
    esac
    env $env timeout -k 10 120 $B > $O/${v}_$r.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v', $r, round(d['ms_per_step']*1e3,2), 'us/iter; sweep', round(d['roofline']['avg_launch_ms']*1e3,2), 'us; pipe', d['sweep_path']['pipe'], 'paired', d['sweep_path']['paired'])"
  done
done
