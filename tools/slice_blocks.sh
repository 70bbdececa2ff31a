#!/bin/bash
# Per-block trace of the fastest and slowest 8-GPU slices (0/8, 7/8) of the 500k grid: the
# producer/consumer default and the grouped-lane form, separate launches (per-block statistics).
set -e -o pipefail
O=gpurun_out/${1:-sblk}
mkdir -p $O
T="timeout -k 10 120 python3 tools/trace_probe.py --n-lam 500000 --blocks --iters 20"
for r in 0 7; do
  FREI_HIP_LIB=abv/trace.so FREI_CHAIN=0 $T --slice $r/8 2>/dev/null > $O/slice_${r}_pipe.txt; cat $O/slice_${r}_pipe.txt
  FREI_HIP_LIB=abv/trace.so FREI_CHAIN=0 FREI_PIPE=0 $T --slice $r/8 2>/dev/null > $O/slice_${r}_grp.txt; cat $O/slice_${r}_grp.txt
done
