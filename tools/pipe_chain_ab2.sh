#!/bin/bash
# Chained producer/consumer sweep with one layer per update block: chain tests, trace, and the
# alternating bench A/B at the 8-GPU slice (pipe separate / pipe chained / grouped chained).
set -e -o pipefail
O=gpurun_out/${1:-pchain}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
T="timeout -k 10 120 python3 tools/trace_probe.py --n-lam 62500"
FREI_HIP_LIB=abv/trace.so FREI_PIPE=4 FREI_CHAIN=2 $T 2>/dev/null > $O/t_pipe_chain.txt; echo "== pipe chain"; cat $O/t_pipe_chain.txt
B="python3 bench.py --n-lam 62500 --steps 40 --warmup 5 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry"
for r in 1 2 3; do
  for cfg in "-1 1" "-1 2" "0 1"; do
    set -- $cfg
    FREI_PIPE=$1 FREI_CHAIN=$2 timeout -k 10 120 $B > $O/b_$1_$2_$r.json 2>/dev/null
    FREI_PIPE=$1 FREI_CHAIN=$2 timeout -k 10 120 $B --force-comm > $O/bp_$1_$2_$r.json 2>/dev/null
    python3 -c "import json; f=lambda n: json.load(open('$O/'+n+'_$1_$2_$r.json')); print('pipe $1 chain $2', $r, round(f('b')['ms_per_step']*1e3,2), 'us/iter; p2p', round(f('bp')['ms_per_step']*1e3,2))"
  done
done
