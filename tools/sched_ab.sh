#!/bin/bash
# LLVM scheduling strategies for the whole kernel file at 500k: default vs max-ILP vs
# max-memory-clause, interleaved.  gpurun_out/sched.
set -o pipefail
O=gpurun_out/sched
mkdir -p $O
timeout -k 10 300 python -u tools/ab_sweep.py --n-lam=500000 --rounds=7 --iters=8 \
  base=frei_amd/libfrei_hip.so ilp=tools/ab_ilp.so mem=tools/ab_memclause.so base2=frei_amd/libfrei_hip.so ilp2=tools/ab_ilp.so mem2=tools/ab_memclause.so > $O/ab.txt 2>&1 || exit $?
grep -o "^.*sweep median [0-9.]* ms\|T-P iteration median [0-9.]* ms" $O/ab.txt | paste - -
