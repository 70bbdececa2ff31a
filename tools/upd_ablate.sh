#!/bin/bash
# Update-kernel ablations at the 8-GPU slice: full vs no next-sweep record (FREI_UPD_NOSETUP) vs an
# empty update kernel (FREI_UPD_EMPTY; results wrong, timing only).  gpurun_out/abl.
set -o pipefail
O=gpurun_out/abl
mkdir -p $O
L=frei_amd/libfrei_hip.so
for n in 62500; do
  timeout -k 10 240 python -u tools/ab_sweep.py --n-lam=$n --rounds=9 --iters=16 \
    full=$L nosetup=tools/ab_nosetup.so empty=tools/ab_empty.so full2=$L > $O/ab_$n.txt 2>&1 || exit $?
  grep -o "^.*sweep median [0-9.]* ms\|T-P iteration median [0-9.]* ms" $O/ab_$n.txt | paste - -
done
