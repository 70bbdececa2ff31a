#!/bin/bash
# Producer/consumer sweep at the 8-GPU slice: role layout (consumers on one SIMD vs rotated) and
# consumer priority, in-kernel trace (FREI_TRACE variants), alternating, then the parity tests
# of the pipe with the rotated layout.
set -e -o pipefail
O=gpurun_out/${1:-piperot}
mkdir -p $O
export FREI_PIPE=4 FREI_CHAIN=0
T="timeout -k 10 120 python3 tools/trace_probe.py --n-lam 62500"
for r in 1 2; do
  for v in trace trace_rot trace_rotprio trace_prio; do
    FREI_HIP_LIB=abv/$v.so $T 2>/dev/null > $O/${v}_$r.txt
    echo "== $v $r"; grep -A3 "kind" $O/${v}_$r.txt | head -3; grep "half" $O/${v}_$r.txt
  done
done
