#!/bin/bash
# Write-through (agent-scope sc1) flux stores (abv/wt2.so, FREI_WT_STORE=2) vs plain stores: chained
# 62.5k slice (trace + bench, alternating) and the 500k bench.
set -e -o pipefail
O=gpurun_out/${1:-wt2}
mkdir -p $O
export FREI_CHAIN=1
T="timeout -k 10 120 python3 tools/trace_probe.py --n-lam 62500"
for lib in trace trace_wt2; do
  FREI_HIP_LIB=abv/$lib.so $T 2>/dev/null > $O/t_$lib.txt; echo "== $lib"; grep -A4 "update_fused', 'chain" $O/t_$lib.txt
done
B="python3 bench.py --steps 40 --warmup 5 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry"
for r in 1 2 3; do
  for lib in default wt2; do
    if [ $lib = default ]; then unset FREI_HIP_LIB; else export FREI_HIP_LIB=abv/$lib.so; fi
    timeout -k 10 120 $B --n-lam 62500 > $O/b_${lib}_$r.json 2>/dev/null
    timeout -k 10 120 $B --n-lam 62500 --force-comm > $O/bp_${lib}_$r.json 2>/dev/null
    timeout -k 10 120 $B --steps 20 > $O/b500_${lib}_$r.json 2>/dev/null
    python3 -c "import json; f=lambda n: json.load(open('$O/'+n+'_${lib}_$r.json')); print('$lib', $r, '62.5k', round(f('b')['ms_per_step']*1e3,2), 'p2p', round(f('bp')['ms_per_step']*1e3,2), '500k', round(f('b500')['ms_per_step']*1e3,2), 'sweep', round(f('b500')['roofline']['avg_launch_ms']*1e3,2))"
  done
done
unset FREI_HIP_LIB
