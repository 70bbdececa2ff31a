#!/bin/bash
# (current, pre-fix) x (forced P2P, no exchange) at 125k, alternated, two rounds.  gpurun_out/p2pi.
set -o pipefail
O=gpurun_out/p2pi
mkdir -p $O
B="python3 bench.py --steps 30 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --n-lam 125000"
for r in 1 2; do
  for v in cur prefix; do
    lib=frei_amd/libfrei_hip.so; [ $v = prefix ] && lib=tools/ab_prefix.so
    for m in none p2p; do
      x=""; [ $m = p2p ] && x="--force-comm"
      FREI_HIP_LIB=$lib timeout -k 10 120 $B $x > $O/${v}_${m}_${r}.json 2>/dev/null || exit $?
      python3 -c "import json; d=json.load(open('$O/${v}_${m}_${r}.json')); print('$v $m $r', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
    done
  done
done
