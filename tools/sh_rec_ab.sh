#!/bin/bash
# LDS step records with in-sweep records (FREI_SHARED_MAX_BLOCKS large) vs the default global
# records at the 2-GPU slice and the full size.  gpurun_out/shrec.
set -o pipefail
O=gpurun_out/shrec
mkdir -p $O
L=frei_amd/libfrei_hip.so
for n in 250000 500000; do
  timeout -k 10 300 python -u tools/ab_sweep.py --n-lam=$n --rounds=9 --iters=8 \
    base=$L shrec=$L@FREI_SHARED_MAX_BLOCKS=100000 base2=$L shrec2=$L@FREI_SHARED_MAX_BLOCKS=100000 > $O/ab_$n.txt 2>&1 || exit $?
  grep -o "^.*sweep median [0-9.]* ms\|T-P iteration median [0-9.]* ms" $O/ab_$n.txt | paste - -
done
