#!/bin/bash
# Producer/consumer vs grouped-lane sweep across small slice sizes (interleaved A/B, one process
# per size).  Outputs under gpurun_out/psize.
set -o pipefail
O=gpurun_out/psize
mkdir -p $O
L=frei_amd/libfrei_hip.so
for n in 31250 47000 55000 62500 70000 78000 94000; do
  timeout -k 10 200 python -u tools/ab_sweep.py --n-lam=$n --rounds=7 --iters=8 \
    grp=$L@FREI_PIPE=0 p4=$L@FREI_PIPE=4 p2=$L@FREI_PIPE=2 p1=$L@FREI_PIPE=1 > $O/ab_$n.txt 2>&1 || exit $?
  cat $O/ab_$n.txt
done
