#!/bin/bash
# Sweep A/B of the current build against abv/old.so at the 8-GPU slice (62.5k, default form:
# producer/consumer) and at 500k (one-lane), interleaved in one process per size.
set -e -o pipefail
O=${1:-gpurun_out/valu}
mkdir -p $O
L=frei_amd/libfrei_hip.so
B=abv/old.so
timeout -k 10 240 python3 tools/ab_sweep.py --n-lam=62500 --rounds=11 --iters=8 \
  old=$B new=$L old2=$B new2=$L > $O/ab_62500.txt
cat $O/ab_62500.txt
timeout -k 10 300 python3 tools/ab_sweep.py --n-lam=500000 --rounds=9 --iters=4 \
  old=$B new=$L old2=$B new2=$L > $O/ab_500000.txt
cat $O/ab_500000.txt
