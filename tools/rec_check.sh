#!/bin/bash
# Step records formed in the sweep (FREI_REC_SWEEP=1) vs written by the update kernel (0):
# GPU test suite, then interleaved A/B of the T-P iteration at the 8/4-GPU slices and 500k.
# gpurun_out/rec.
set -o pipefail
O=gpurun_out/rec
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=frei_amd/libfrei_hip.so
for n in 62500 125000 500000; do
  timeout -k 10 240 python -u tools/ab_sweep.py --n-lam=$n --rounds=9 --iters=16 \
    rec0=$L@FREI_REC_SWEEP=0 rec1=$L@FREI_REC_SWEEP=1 rec0b=$L@FREI_REC_SWEEP=0 rec1b=$L@FREI_REC_SWEEP=1 > $O/ab_$n.txt 2>&1 || exit $?
  grep -o "^.*sweep median [0-9.]* ms\|T-P iteration median [0-9.]* ms" $O/ab_$n.txt | paste - -
done
