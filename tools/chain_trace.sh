#!/bin/bash
# Wave -> SIMD map of 1024/512/256-thread blocks, then the chained launch's in-kernel trace at the
# 8-GPU slice (4- and 8-wave grouped blocks, with and without the one-rank P2P exchange).
set -e -o pipefail
O=gpurun_out/${1:-ctrace}
mkdir -p $O
timeout -k 10 60 ./tools/simd_map > $O/simd_map.txt 2>&1; cat $O/simd_map.txt
T="timeout -k 10 120 python3 tools/trace_probe.py"
for w in 4 8; do
  FREI_HIP_LIB=abv/trace.so FREI_CHAIN=1 FREI_GROUP_WAVES=$w $T --n-lam 62500 > $O/t_w$w.txt 2>&1
  echo "== chain, waves $w"; cat $O/t_w$w.txt
  FREI_HIP_LIB=abv/trace.so FREI_CHAIN=1 FREI_GROUP_WAVES=$w $T --n-lam 62500 --p2p > $O/tp_w$w.txt 2>&1
  echo "== chain p2p, waves $w"; cat $O/tp_w$w.txt
done
