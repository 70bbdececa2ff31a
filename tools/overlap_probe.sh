#!/bin/bash
# 500k one-lane sweep: full vs memory-only (trivial arithmetic) vs cache-only (table and stale loads
# from a 32 KB cache-resident region; same instructions) builds, interleaved.  gpurun_out/ovl.
set -o pipefail
O=gpurun_out/ovl
mkdir -p $O
L=frei_amd/libfrei_hip.so
timeout -k 10 300 python -u tools/ab_sweep.py --n-lam=500000 --rounds=7 --iters=4 \
  full=$L mem=tools/ab_memonly.so cache=tools/ab_cacheonly.so > $O/ab_500000.txt 2>&1 || exit $?
cat $O/ab_500000.txt
