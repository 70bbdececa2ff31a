#!/bin/bash
# Chained launches, one-lane polling: bit-identity tests, chained trace at the 8-GPU slice (4- and
# 8-wave blocks, with and without the one-rank P2P exchange) and alternating bench A/B.
set -e -o pipefail
O=gpurun_out/${1:-chain3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
T="timeout -k 10 120 python3 tools/trace_probe.py --n-lam 62500"
for w in 4 8; do
  FREI_HIP_LIB=abv/trace.so FREI_CHAIN=1 FREI_GROUP_WAVES=$w $T 2>/dev/null > $O/t_w$w.txt; echo "== waves $w"; grep -A3 "update_fused', 'chain" $O/t_w$w.txt
  FREI_HIP_LIB=abv/trace.so FREI_CHAIN=1 FREI_GROUP_WAVES=$w $T --p2p 2>/dev/null > $O/tp_w$w.txt; echo "== waves $w p2p"; grep -A3 "update_fused', 'chain" $O/tp_w$w.txt
done
B="python3 bench.py --n-lam 62500 --steps 40 --warmup 5 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry"
for r in 1 2 3; do
  for cfg in "0 4" "1 4" "1 8"; do
    set -- $cfg
    FREI_CHAIN=$1 FREI_GROUP_WAVES=$2 timeout -k 10 120 $B > $O/b_$1_$2_$r.json 2>/dev/null
    FREI_CHAIN=$1 FREI_GROUP_WAVES=$2 timeout -k 10 120 $B --force-comm > $O/bp_$1_$2_$r.json 2>/dev/null
    python3 -c "import json; f=lambda n: json.load(open('$O/'+n+'_$1_$2_$r.json')); print('chain $1 waves $2', $r, round(f('b')['ms_per_step']*1e3,2), 'us/iter; p2p', round(f('bp')['ms_per_step']*1e3,2))"
  done
done
