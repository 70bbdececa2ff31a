#!/bin/bash
# Chained launches with per-layer convergence granules: bit-identity tests, the chained trace and
# bench lines at the 8-GPU slice (chain off / on alternating, with and without one-rank P2P).
set -e -o pipefail
O=gpurun_out/${1:-chain2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py -k "chain or grouped_lane" -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
T="timeout -k 10 120 python3 tools/trace_probe.py"
FREI_HIP_LIB=abv/trace.so FREI_CHAIN=1 $T --n-lam 62500 2>/dev/null | grep -v "launch type \['update_fused'\]\|^     update_fused: first entry   0.00" > $O/t_ch1.txt; cat $O/t_ch1.txt
FREI_HIP_LIB=abv/trace.so FREI_CHAIN=1 $T --n-lam 62500 --p2p 2>/dev/null > $O/tp_ch1.txt; cat $O/tp_ch1.txt
B="python3 bench.py --n-lam 62500 --steps 40 --warmup 5 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry"
for r in 1 2 3; do
  for ch in 0 1; do
    FREI_CHAIN=$ch timeout -k 10 120 $B > $O/b_ch${ch}_$r.json 2>/dev/null
    FREI_CHAIN=$ch timeout -k 10 120 $B --force-comm > $O/bp_ch${ch}_$r.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/b_ch${ch}_$r.json')); e=json.load(open('$O/bp_ch${ch}_$r.json')); print('chain $ch', $r, round(d['ms_per_step']*1e3,2), 'us/iter; p2p', round(e['ms_per_step']*1e3,2))"
  done
done
