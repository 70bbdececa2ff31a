#!/bin/bash
# Chained launches (FREI_CHAIN=1): bit-identity tests, then the in-kernel trace and bench lines at
# the 8-GPU slice, chain off / on alternating, with and without the one-rank P2P exchange.
set -e -o pipefail
O=gpurun_out/${1:-chain}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
T="timeout -k 10 120 python3 tools/trace_probe.py"
for ch in 0 1; do
  FREI_HIP_LIB=abv/trace.so FREI_CHAIN=$ch $T --n-lam 62500 > $O/t_ch${ch}.txt 2>&1
  echo "== chain $ch"; cat $O/t_ch${ch}.txt
done
B="python3 bench.py --n-lam 62500 --steps 40 --warmup 5 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry"
for r in 1 2 3; do
  for ch in 0 1; do
    FREI_CHAIN=$ch timeout -k 10 120 $B > $O/b_ch${ch}_$r.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/b_ch${ch}_$r.json')); print('chain $ch', $r, round(d['ms_per_step']*1e3,2), 'us/iter')"
    FREI_CHAIN=$ch timeout -k 10 120 $B --force-comm > $O/bp_ch${ch}_$r.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/bp_ch${ch}_$r.json')); print('chain $ch p2p', $r, round(d['ms_per_step']*1e3,2), 'us/iter')"
  done
done
