#!/bin/bash
# Records formed in the sweep vs written by the update: interleaved A/B only.  gpurun_out/rec2.
set -o pipefail
O=gpurun_out/rec2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "records or pipe" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=frei_amd/libfrei_hip.so
for n in 62500 125000; do
  timeout -k 10 240 python -u tools/ab_sweep.py --n-lam=$n --rounds=9 --iters=16 \
    rec0=$L@FREI_REC_SWEEP=0 rec1=$L@FREI_REC_SWEEP=1 rec0b=$L@FREI_REC_SWEEP=0 rec1b=$L@FREI_REC_SWEEP=1 > $O/ab_$n.txt 2>&1 || exit $?
  grep -o "^.*sweep median [0-9.]* ms\|T-P iteration median [0-9.]* ms" $O/ab_$n.txt | paste - -
done
