#!/bin/bash
# Whole GPU suite + bench on the current tree.
set -o pipefail
O=gpurun_out/${1:-r04c10}
mkdir -p $O
FREI_PARITY_JSON=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 700 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -1 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  timeout -k 10 120 python3 bench.py $B > $O/b_$rep.json 2> $O/b_$rep.err || { echo "bench failed"; exit 3; }
  python3 -c "import json; a=json.load(open('$O/b_$rep.json')); print($rep, '500k %.4f ms sweep %.2f us frac %.3f' % (a['ms_per_step'], a['roofline']['avg_launch_ms']*1e3, a['roofline']['frac']), flush=True)" | tee -a $O/summary.txt
done
