#!/bin/bash
# A/B: the sweep's load ring with the refill ordered after the consuming opacity (HEAD build,
# FREI_RING_DEP) vs the previous tree's build (ablib/base.so), interleaved at 500k and at the
# 8-GPU slice; then the sweep parity / bit-identity tests on the new build.
set -o pipefail
O=gpurun_out/${1:-r04ring}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  for t in ringdep2 base; do
    L="FREI_HIP_LIB=ablib/$t.so"
    env $L timeout -k 10 120 python3 bench.py $B > $O/${t}_500k_$rep.json 2> /dev/null || { echo "bench $t failed"; exit 3; }
    env $L timeout -k 10 120 python3 bench.py $B --rad-eq-max 1 --steps 40 --force-comm --lam-slice 0:62500 > $O/${t}_s0_$rep.json 2> /dev/null || { echo "bench slice $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_500k_$rep.json')); b=json.load(open('$O/${t}_s0_$rep.json')); print('$t', $rep, '500k %.4f ms sweep %.2f us' % (a['ms_per_step'], a['roofline']['avg_launch_ms']*1e3), 'slice0 %.2f us' % (b['ms_per_step']*1e3), flush=True)" | tee -a $O/summary.txt
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_update.py tests/test_gpu_chain.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
grep -E "FAILED" $O/pytest.log | head; tail -1 $O/pytest.log
