#!/bin/bash
# Producer/consumer sweep: bit-identity tests, then interleaved A/B timing against the one-lane and
# grouped-lane forms at slice sizes given as arguments (default: the 8/4-GPU slices).
# Outputs under gpurun_out/pipe.
set -o pipefail
O=gpurun_out/pipe
mkdir -p $O
L=frei_amd/libfrei_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "pipe or high_albedo" > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in ${@:-62500 125000}; do
  timeout -k 10 240 python -u tools/ab_sweep.py --n-lam=$n --rounds=7 --iters=8 \
    grp=$L@FREI_PIPE=0 p4pf1=$L@FREI_PIPE=4,FREI_PIPE_PF=1 p4=$L@FREI_PIPE=4 \
    p2=$L@FREI_PIPE=2 p1=$L@FREI_PIPE=1 > $O/ab_$n.txt 2>&1 || exit $?
  cat $O/ab_$n.txt
done
