#!/bin/bash
# Forced one-rank P2P at 250k: with / without the push (ablation), and no exchange, alternated.
set -o pipefail
O=gpurun_out/p2pp
mkdir -p $O
B="python3 bench.py --steps 30 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --n-lam 250000"
for r in 1 2 3; do
  for v in none p2p nopush; do
    lib=frei_amd/libfrei_hip.so; x="--force-comm"
    [ $v = nopush ] && lib=tools/ab_nopush.so; [ $v = none ] && x=""
    FREI_HIP_LIB=$lib timeout -k 10 120 $B $x > $O/${v}_${r}.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$O/${v}_${r}.json')); print('$v $r', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
