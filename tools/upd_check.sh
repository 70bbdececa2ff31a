#!/bin/bash
# Update-kernel change A/B: fused-update bit-identity tests, then T-P iteration wall time of the
# previous build vs the current one (interleaved).  gpurun_out/upd.
set -o pipefail
O=gpurun_out/upd
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_update.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 62500 500000; do
  timeout -k 10 240 python -u tools/ab_sweep.py --n-lam=$n --rounds=9 --iters=8 \
    prev=tools/ab_prev.so cur=frei_amd/libfrei_hip.so prev2=tools/ab_prev.so cur2=frei_amd/libfrei_hip.so > $O/ab_$n.txt 2>&1 || exit $?
  grep -o "^.*sweep median [0-9.]* ms\|T-P iteration median [0-9.]* ms" $O/ab_$n.txt | paste - -
done
