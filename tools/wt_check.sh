#!/bin/bash
# Write-through (system-scope) flux stores vs plain stores, interleaved A/B.  gpurun_out/wt.
set -o pipefail
O=gpurun_out/wt
mkdir -p $O
L=frei_amd/libfrei_hip.so
W=tools/ab_wt.so
for n in 62500 500000; do
  timeout -k 10 240 python -u tools/ab_sweep.py --n-lam=$n --rounds=7 --iters=8 \
    base=$L wt=$W base1=$L@FREI_GROUP_Q=1,FREI_PIPE=0 wt1=$W@FREI_GROUP_Q=1,FREI_PIPE=0 > $O/ab_$n.txt 2>&1 || exit $?
  cat $O/ab_$n.txt
done
