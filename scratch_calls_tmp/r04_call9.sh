#!/bin/bash
# Two wavelengths per lane: its bitwise/rounding tests first (stop on any failure), then
# lam2 (auto) vs one-lane (FREI_LAM2=0) interleaved at 500k, then the whole GPU suite.
set -o pipefail
O=gpurun_out/${1:-r04c9}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lam2.py -v --timeout 240 --timeout-method thread > $O/pytest_lam2.log 2>&1
rc=$?
tail -8 $O/pytest_lam2.log
[ $rc -ne 0 ] && exit $rc
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  for t in lam2 one; do
    if [ $t = lam2 ]; then E="FREI_LAM2=-1"; else E="FREI_LAM2=0"; fi
    env $E timeout -k 10 120 python3 bench.py $B > $O/${t}_500k_$rep.json 2> $O/${t}_500k_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_500k_$rep.json')); print('$t', $rep, '500k %.4f ms sweep %.2f us frac %.3f' % (a['ms_per_step'], a['roofline']['avg_launch_ms']*1e3, a['roofline']['frac']), flush=True)" | tee -a $O/summary.txt
  done
done
FREI_PARITY_JSON=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 700 --timeout-method thread > $O/pytest.log 2>&1
grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -1 $O/pytest.log
