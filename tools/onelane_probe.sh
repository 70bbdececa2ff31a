#!/bin/bash
# One-lane sweep at the 8-GPU slice (one wave per SIMD): full, cache-only (FREI_CACHEONLY: same
# instructions, loads from a cache-resident 32 KB) and memory-only (FREI_MEMONLY: same traffic,
# trivial arithmetic) trace builds at prefetch depth 2 and 4, and the prefetch distance 8 / 16.
set -e -o pipefail
O=gpurun_out/${1:-onelane}
mkdir -p $O
T="timeout -k 10 120 python3 tools/trace_probe.py --n-lam 62500 --iters 20"
export FREI_GROUP_Q=1 FREI_PIPE=0
for lib in trace trace_co trace_mo; do
  for d in 2 4; do
    FREI_HIP_LIB=abv/$lib.so FREI_PREFETCH_DEPTH=$d $T > $O/${lib}_d$d.txt 2>&1
    echo "== $lib depth $d"; grep -A3 "kind" $O/${lib}_d$d.txt | head -3
  done
done
for pf in 8 16; do
  FREI_HIP_LIB=abv/trace.so FREI_PREFETCH_STEPS=$pf $T > $O/trace_pf$pf.txt 2>&1
  echo "== trace pf $pf"; grep -A3 "kind" $O/trace_pf$pf.txt | head -3
done
