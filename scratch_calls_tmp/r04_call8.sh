#!/bin/bash
# Round-4 tree with the exp-form Planck, the shared coefficient tail, batched update sums and
# progress-ordered issue priority: the GPU suite first, then priority on/off interleaved at
# 500k, then the sweep time per lambda by number of block rounds.
set -o pipefail
O=gpurun_out/${1:-r04c8}
mkdir -p $O
FREI_PARITY_JSON=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 700 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -1 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  for t in cur prio0; do
    if [ $t = cur ]; then E="FREI_SKIP_NOTHING=1"; else E="FREI_HIP_LIB=ablib/prio0.so"; fi
    env $E timeout -k 10 120 python3 bench.py $B > $O/${t}_500k_$rep.json 2> $O/${t}_500k_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_500k_$rep.json')); print('$t', $rep, '500k %.4f ms sweep %.2f us' % (a['ms_per_step'], a['roofline']['avg_launch_ms']*1e3), flush=True)" | tee -a $O/summary.txt
  done
done
bash tools/calls/r04_rounds.sh ${1:-r04c8}/rounds
