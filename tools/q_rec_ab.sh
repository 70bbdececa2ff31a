#!/bin/bash
# Lanes per wavelength with in-sweep records (default): Q=1 vs Q=2 around the pair threshold.
set -o pipefail
O=gpurun_out/qrec
mkdir -p $O
L=frei_amd/libfrei_hip.so
for n in 94000 110000 125000; do
  timeout -k 10 240 python -u tools/ab_sweep.py --n-lam=$n --rounds=9 --iters=16 \
    q1=$L@FREI_GROUP_Q=1,FREI_PIPE=0 q2=$L@FREI_GROUP_Q=2,FREI_PIPE=0 q1b=$L@FREI_GROUP_Q=1,FREI_PIPE=0 q2b=$L@FREI_GROUP_Q=2,FREI_PIPE=0 > $O/ab_$n.txt 2>&1 || exit $?
  echo "n $n"; grep -o "^.*sweep median [0-9.]* ms\|T-P iteration median [0-9.]* ms" $O/ab_$n.txt | paste - -
done
