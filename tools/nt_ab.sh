#!/bin/bash
# Nontemporal table-row loads (FREI_NT=1) vs plain, interleaved, at 500k and 250k.  gpurun_out/nt.
set -o pipefail
O=gpurun_out/nt
mkdir -p $O
for n in 500000 250000; do
  timeout -k 10 300 python -u tools/ab_sweep.py --n-lam=$n --rounds=9 --iters=8 \
    base=frei_amd/libfrei_hip.so nt=tools/ab_nt.so base2=frei_amd/libfrei_hip.so nt2=tools/ab_nt.so > $O/ab_$n.txt 2>&1 || exit $?
  grep -o "^.*sweep median [0-9.]* ms\|T-P iteration median [0-9.]* ms" $O/ab_$n.txt | paste - -
done
