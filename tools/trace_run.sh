#!/bin/bash
# In-kernel trace of the T-P half-iteration (tools/trace_probe.py, abv/trace.so = FREI_TRACE build)
# at the 8-GPU slice with and without the one-rank P2P exchange, and at 500k.
set -e -o pipefail
O=gpurun_out/${1:-trace}
mkdir -p $O
export FREI_HIP_LIB=abv/trace.so
timeout -k 10 120 python3 tools/trace_probe.py --n-lam 62500 > $O/t62500.txt 2>&1
timeout -k 10 120 python3 tools/trace_probe.py --n-lam 62500 --p2p > $O/t62500_p2p.txt 2>&1
timeout -k 10 120 python3 tools/trace_probe.py --n-lam 500000 --iters 20 > $O/t500000.txt 2>&1
cat $O/t62500.txt $O/t62500_p2p.txt $O/t500000.txt
