#!/bin/bash
# C5 batched throughput with step records formed in the sweep (1) or by the update (0), alternated.
set -o pipefail
O=gpurun_out/c5rec
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    FREI_REC_SWEEP=$v timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-binning --no-per-species --no-chemistry --no-cpu-baseline --c5-steps 10 > $O/r${v}_$r.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$O/r${v}_$r.json'))['c5_batched']; print('rec', $v, $r, d['updates_per_s'], d['ms_per_step'], d['rad_eq']['wall_s'])"
  done
done
