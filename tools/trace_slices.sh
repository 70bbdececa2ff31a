#!/bin/bash
# In-kernel trace (FREI_TRACE build abv/trace.so) of the 8-GPU slices: the full-range 62.5k grid
# with the per-block distribution, then every rank's slice r/8 of the 500k grid on this one GPU.
set -e -o pipefail
O=gpurun_out/${1:-trace2}
mkdir -p $O
export FREI_HIP_LIB=abv/trace.so
timeout -k 10 120 python3 tools/trace_probe.py --n-lam 62500 --blocks > $O/t62500_blocks.txt 2>&1
cat $O/t62500_blocks.txt
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 python3 tools/trace_probe.py --n-lam 500000 --slice $r/8 --blocks > $O/slice_$r.txt 2>&1
  cat $O/slice_$r.txt
done
