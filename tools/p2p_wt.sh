#!/bin/bash
# Forced one-rank P2P at 250k / 125k: plain vs write-through flux stores, with and without the
# exchange, alternated.  gpurun_out/p2pwt.
set -o pipefail
O=gpurun_out/p2pwt
mkdir -p $O
B="python3 bench.py --steps 30 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1"
for r in 1 2; do
  for n in 250000 125000; do
    for v in cur wt; do
      lib=frei_amd/libfrei_hip.so; [ $v = wt ] && lib=tools/ab_wt.so
      for m in none p2p; do
        x=""; [ $m = p2p ] && x="--force-comm"
        FREI_HIP_LIB=$lib timeout -k 10 120 $B --n-lam $n $x > $O/${v}_${m}_${n}_${r}.json 2>/dev/null || exit $?
        python3 -c "import json; d=json.load(open('$O/${v}_${m}_${n}_${r}.json')); print('$v $m $n $r', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
      done
    done
  done
done
