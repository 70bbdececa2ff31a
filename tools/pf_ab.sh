#!/bin/bash
# Sweep A/B at the 8-GPU slice (62.5k) and at 500k: the previous build (abv/old.so) against the
# current one (load ring without latch drains), at prefetch distances 2 / 8 / 16 steps and in
# the default forms; interleaved in one process per size (tools/ab_sweep.py).
set -e -o pipefail
O=${1:-gpurun_out/pf}
mkdir -p $O
L=frei_amd/libfrei_hip.so
B=abv/old.so
one="FREI_GROUP_Q=1,FREI_PIPE=0"
timeout -k 10 240 python3 tools/ab_sweep.py --n-lam=62500 --rounds=9 --iters=8 \
  old_default=$B new_default=$L "old_one=$B@$one" "one=$L@$one" \
  "one_pf8=$L@$one,FREI_PREFETCH_STEPS=8" "one_pf16=$L@$one,FREI_PREFETCH_STEPS=16" \
  "one_d4=$L@$one,FREI_PREFETCH_DEPTH=4" \
  "one_d4_pf8=$L@$one,FREI_PREFETCH_DEPTH=4,FREI_PREFETCH_STEPS=8" \
  "one_d4_pf16=$L@$one,FREI_PREFETCH_DEPTH=4,FREI_PREFETCH_STEPS=16" > $O/ab_62500.txt
cat $O/ab_62500.txt
timeout -k 10 300 python3 tools/ab_sweep.py --n-lam=500000 --rounds=7 --iters=4 \
  old=$B default=$L "pf8=$L@FREI_PREFETCH_STEPS=8" "d4=$L@FREI_PREFETCH_DEPTH=4" \
  "d4_pf8=$L@FREI_PREFETCH_DEPTH=4,FREI_PREFETCH_STEPS=8" > $O/ab_500000.txt
cat $O/ab_500000.txt
