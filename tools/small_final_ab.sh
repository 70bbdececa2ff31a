#!/bin/bash
# 62.5k / 55k: producer/consumer (records by the update) vs grouped-lane with in-sweep records vs
# producer/consumer with in-sweep records, interleaved.  gpurun_out/sfa.
set -o pipefail
O=gpurun_out/sfa
mkdir -p $O
L=frei_amd/libfrei_hip.so
for n in 62500 55000; do
  timeout -k 10 240 python -u tools/ab_sweep.py --n-lam=$n --rounds=9 --iters=16 \
    pipe=$L grp_rec=$L@FREI_PIPE=0 pipe_rec=$L@FREI_REC_SWEEP=1 pipe2=$L grp_rec2=$L@FREI_PIPE=0 > $O/ab_$n.txt 2>&1 || exit $?
  grep -o "^.*sweep median [0-9.]* ms\|T-P iteration median [0-9.]* ms" $O/ab_$n.txt | paste - -
done
