#!/bin/bash
# Default bench line three times on one box (run-to-run spread).  gpurun_out/repeat.
set -o pipefail
O=gpurun_out/repeat
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 400 python3 bench.py > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print($i, d['value'], d['ms_per_step'], d['roofline']['frac'], d['c5_batched']['rad_eq']['converged_rank0'])"
done
