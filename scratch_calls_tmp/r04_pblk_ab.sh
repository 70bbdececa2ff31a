#!/bin/bash
# Partial sums block-major (each sweep block writes whole lines; pblk) vs the step-major layout
# (base), interleaved at 500k and at the 2- and 8-GPU slices; then the whole GPU suite.
set -o pipefail
O=gpurun_out/${1:-r04pblk}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  for t in pblk base; do
    E="FREI_HIP_LIB=ablib/$t.so"
    env $E timeout -k 10 120 python3 bench.py $B > $O/${t}_500k_$rep.json 2> /dev/null || { echo "bench $t failed"; exit 3; }
    env $E timeout -k 10 120 python3 bench.py $B --rad-eq-max 1 --force-comm --lam-slice 0:250000 > $O/${t}_s2_$rep.json 2> /dev/null || { echo "bench s2 $t failed"; exit 3; }
    env $E timeout -k 10 120 python3 bench.py $B --rad-eq-max 1 --steps 40 --force-comm --lam-slice 0:62500 > $O/${t}_s8_$rep.json 2> /dev/null || { echo "bench s8 $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_500k_$rep.json')); b=json.load(open('$O/${t}_s2_$rep.json')); c=json.load(open('$O/${t}_s8_$rep.json')); print('$t', $rep, '500k %.4f ms' % a['ms_per_step'], '250k %.2f us' % (b['ms_per_step']*1e3), '62.5k %.2f us' % (c['ms_per_step']*1e3), flush=True)" | tee -a $O/summary.txt
  done
done
FREI_PARITY_JSON=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 700 --timeout-method thread > $O/pytest.log 2>&1
grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -1 $O/pytest.log
