#!/bin/bash
# Update-kernel ablations at 500k (timing only; the ablated builds give wrong results).  gpurun_out/abl5.
set -o pipefail
O=gpurun_out/abl5
mkdir -p $O
L=frei_amd/libfrei_hip.so
timeout -k 10 300 python -u tools/ab_sweep.py --n-lam=500000 --rounds=7 --iters=8 \
  full=$L nosum=tools/ab_NOSUM.so nodt=tools/ab_NODT.so nosetup=tools/ab_NOSETUP.so empty=tools/ab_EMPTY.so > $O/ab.txt 2>&1 || exit $?
grep -o "^.*sweep median [0-9.]* ms\|T-P iteration median [0-9.]* ms" $O/ab.txt | paste - -
