#!/bin/bash
# In-kernel trace (FREI_TRACE build abv/trace.so) of the 8-GPU slice: the full-range 62.5k grid
# with the per-block distribution, by blocks-per-CU cap (FREI_SWEEP_LDS_KB) and sweep form, then
# every rank's slice r/8 of the 500k grid on this one GPU.
set -e -o pipefail
O=gpurun_out/${1:-trace2}
mkdir -p $O
export FREI_HIP_LIB=abv/trace.so
T="timeout -k 10 120 python3 tools/trace_probe.py"
$T --n-lam 62500 --blocks > $O/t62500_blocks.txt 2>&1; cat $O/t62500_blocks.txt
FREI_SWEEP_LDS_KB=56 $T --n-lam 62500 --blocks > $O/t62500_lds56.txt 2>&1; cat $O/t62500_lds56.txt
FREI_GROUP_Q=1 FREI_PIPE=0 $T --n-lam 62500 --blocks > $O/t62500_one.txt 2>&1; cat $O/t62500_one.txt
FREI_GROUP_Q=1 FREI_PIPE=0 FREI_SWEEP_LDS_KB=96 $T --n-lam 62500 --blocks > $O/t62500_one_lds96.txt 2>&1; cat $O/t62500_one_lds96.txt
FREI_PIPE=4 $T --n-lam 62500 --blocks > $O/t62500_pipe.txt 2>&1; cat $O/t62500_pipe.txt
for r in 0 3 7; do
  $T --n-lam 500000 --slice $r/8 > $O/slice_$r.txt 2>&1; cat $O/slice_$r.txt
done
