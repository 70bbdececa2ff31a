#!/bin/bash
# Reproduce the C5 iteration-count anomaly: bench.py with different legs before C5.  gpurun_out/c5r.
set -o pipefail
O=gpurun_out/c5r
mkdir -p $O
run() {   # name, extra args
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "${@:2}" > $O/$1.json 2>$O/$1.err || return $?
  python3 -c "import json; d=json.load(open('$O/$1.json'))['c5_batched']['rad_eq']; print('$1', d['iterations_min'], d['iterations_max'], d['converged_rank0'])"
}
run full && run full_again && run c5only --no-binning --no-per-species --no-chemistry \
  && run nobin --no-binning && run nochem --no-chemistry && run nops --no-per-species
