#!/bin/bash
# Round-4 GPU call: lean-lite (HEAD, premultiplied coefficients only) vs the literal form at
# 500k and at the 8-GPU slice (62.5k, one-rank P2P), interleaved; then the tests that failed with
# the identity-based lean form.
set -o pipefail
O=gpurun_out/${1:-r04c7}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  for t in lite literal; do
    if [ $t = lite ]; then L=""; else L="FREI_HIP_LIB=abtree/nolean.so"; fi
    env $L timeout -k 10 120 python3 bench.py $B > $O/${t}_500k_$rep.json 2> /dev/null || { echo "bench $t failed"; exit 3; }
    env $L timeout -k 10 120 python3 bench.py $B --rad-eq-max 1 --steps 40 --force-comm --lam-slice 0:62500 > $O/${t}_s0_$rep.json 2> /dev/null || { echo "bench slice $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_500k_$rep.json')); b=json.load(open('$O/${t}_s0_$rep.json')); print('$t', $rep, '500k %.4f ms' % a['ms_per_step'], 'slice0 %.2f us' % (b['ms_per_step']*1e3), flush=True)" | tee -a $O/summary.txt
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_c4.py tests/test_gpu_chemistry_provider.py tests/test_gpu_parity.py -v --timeout 700 --timeout-method thread > $O/pytest.log 2>&1
grep -E "FAILED" $O/pytest.log | head; tail -1 $O/pytest.log
