#!/bin/bash
# Forced-P2P step time at 125k: current vs the race fix with one piece reverted.  gpurun_out/p2pb.
set -o pipefail
O=gpurun_out/p2pb
mkdir -p $O
B="python3 bench.py --steps 30 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --n-lam 125000 --force-comm"
for r in 1 2; do
  for v in cur prefix mbox ticks h2d; do
    lib=tools/ab_$v.so; [ $v = cur ] && lib=frei_amd/libfrei_hip.so
    FREI_HIP_LIB=$lib timeout -k 10 120 $B > $O/${v}_${r}.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$O/${v}_${r}.json')); print('$v $r', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
