#!/bin/bash
# Small-slice forms after the load-ring fix (current build) against the previous build
# (abv/old.so): producer/consumer (default at 62.5k) and the grouped-lane forms Q = 2, 4.
set -e -o pipefail
O=${1:-gpurun_out/grp}
mkdir -p $O
L=frei_amd/libfrei_hip.so
B=abv/old.so
for n in 62500 47000 94000; do
  timeout -k 10 240 python3 tools/ab_sweep.py --n-lam=$n --rounds=9 --iters=8 \
    old_default=$B default=$L "old_q2=$B@FREI_PIPE=0,FREI_GROUP_Q=2" "q2=$L@FREI_PIPE=0,FREI_GROUP_Q=2" \
    "old_q4=$B@FREI_PIPE=0,FREI_GROUP_Q=4" "q4=$L@FREI_PIPE=0,FREI_GROUP_Q=4" > $O/ab_$n.txt
  cat $O/ab_$n.txt
done
