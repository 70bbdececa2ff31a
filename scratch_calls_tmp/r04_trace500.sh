#!/bin/bash
# Where a 500k T-P half-iteration goes (FREI_TRACE build, in-kernel clock marks).
set -o pipefail
O=gpurun_out/${1:-r04trace}
mkdir -p $O
FREI_HIP_LIB=ablib/trace.so timeout -k 10 200 python3 tools/trace_probe.py --n-lam 500000 --iters 20 --blocks > $O/trace500.txt 2>&1
cat $O/trace500.txt | head -60
