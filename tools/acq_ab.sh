#!/bin/bash
# Cost of the P2P consumer's system-scope acquire (p2p_acquire): bench.py at the 8-GPU slice
# with the one-rank P2P exchange forced on, current build vs abv/noacq.so (FREI_P2P_ACQ=0),
# alternating; and the fused update's duration in a rocprof kernel trace of each.
set -e -o pipefail
O=${1:-gpurun_out/acq}
mkdir -p $O
B="python3 bench.py --n-lam 62500 --steps 40 --warmup 5 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --force-comm"
for r in 1 2 3; do
  for v in acq noacq; do
    if [ $v = noacq ]; then export FREI_HIP_LIB=abv/noacq.so; else unset FREI_HIP_LIB; fi
    timeout -k 10 120 $B > $O/${v}_$r.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v', $r, round(d['ms_per_step']*1e3,2), 'us/iter; sweep', round(d['roofline']['avg_launch_ms']*1e3,2), 'us; exchange wait', round(d['exchange']['avg_ms']*1e3,2), 'us')"
  done
done
unset FREI_HIP_LIB
