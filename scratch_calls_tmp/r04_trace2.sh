#!/bin/bash
# In-kernel trace of the 500k half iteration and of the 8-GPU slice (FREI_TRACE build).
set -o pipefail
O=gpurun_out/${1:-r04tr2}
mkdir -p $O
FREI_HIP_LIB=ablib/trace.so timeout -k 10 200 python3 tools/trace_probe.py --n-lam 500000 --iters 20 > $O/trace500.txt 2>&1
FREI_HIP_LIB=ablib/trace.so timeout -k 10 200 python3 tools/trace_probe.py --n-lam 62500 --p2p --iters 40 > $O/trace62500_p2p.txt 2>&1
head -6 $O/trace500.txt; head -8 $O/trace62500_p2p.txt
