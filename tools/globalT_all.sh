#!/bin/bash
# Per-rank sweep time at the global temperatures for N = 2, 4, 8 (tools/slice_globalT.py).
set -e -o pipefail
O=gpurun_out/${1:-gT}
mkdir -p $O
for n in 2 4 8; do
  timeout -k 10 300 python3 tools/slice_globalT.py --n $n --iters 40 > $O/globalT_$n.txt 2>&1; cat $O/globalT_$n.txt
done
