#!/bin/bash
# C5 iteration-count anomaly: runs with every device buffer pre-filled (FREI_ALLOC_FILL) — zero,
# 0x40 (2.0 doubles), 0xFF (NaN) — alone and after a C3 context.  gpurun_out/c5fill.
set -o pipefail
O=gpurun_out/c5fill
mkdir -p $O
for f in 0 64 255; do
  FREI_ALLOC_FILL=$f timeout -k 10 300 python3 tools/c5_determinism.py 100000 -1.0 0 > $O/alone_$f.txt 2>&1 || exit $?
  echo "fill $f alone: $(tail -1 $O/alone_$f.txt)"
  FREI_ALLOC_FILL=$f timeout -k 10 300 python3 tools/c5_determinism.py 100000 -1.0 0 afterc3 > $O/after_$f.txt 2>&1 || exit $?
  echo "fill $f afterc3: $(tail -1 $O/after_$f.txt)"
done
