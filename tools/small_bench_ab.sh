#!/bin/bash
# bench.py at the 8-GPU slice with the one-rank P2P exchange: producer/consumer (default at the
# time) vs grouped-lane with in-sweep records (FREI_PIPE=0), alternated, three rounds.
set -o pipefail
O=gpurun_out/sba
mkdir -p $O
B="python3 bench.py --steps 40 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --n-lam 62500 --force-comm"
for r in 1 2 3; do
  for v in pipe grp; do
    env=""; [ $v = grp ] && env="FREI_PIPE=0"
    env $env timeout -k 10 120 $B > $O/${v}_${r}.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$O/${v}_${r}.json')); print('$v $r', round(d['ms_per_step'],5), round(d['roofline']['avg_launch_ms'],5), d['sweep_path']['pipe'], d['sweep_path']['paired'])"
  done
done
