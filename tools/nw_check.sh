#!/bin/bash
# Grouped-lane sweep with 8-wave blocks (FREI_GROUP_WAVES=8): the grouped-lane parity tests, then
# the in-kernel trace at the 8-GPU slice (4- vs 8-wave blocks, alternating) and bench lines.
set -e -o pipefail
O=gpurun_out/${1:-nw}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "grouped_lane or pipe_sweep" -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
tail -2 $O/pytest.txt
T="timeout -k 10 120 python3 tools/trace_probe.py"
for r in 1 2; do
  for w in 4 8; do
    FREI_HIP_LIB=abv/trace.so FREI_GROUP_WAVES=$w $T --n-lam 62500 --blocks > $O/t_w${w}_$r.txt 2>&1
    echo "== waves $w run $r"; cat $O/t_w${w}_$r.txt
  done
done
B="python3 bench.py --n-lam 62500 --steps 40 --warmup 5 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry"
for r in 1 2; do
  for w in 4 8; do
    FREI_GROUP_WAVES=$w timeout -k 10 120 $B > $O/b_w${w}_$r.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/b_w${w}_$r.json')); print('waves $w', $r, round(d['ms_per_step']*1e3,2), 'us/iter; sweep', round(d['roofline']['avg_launch_ms']*1e3,2))"
    FREI_GROUP_WAVES=$w timeout -k 10 120 $B --force-comm > $O/bp_w${w}_$r.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/bp_w${w}_$r.json')); print('waves $w p2p', $r, round(d['ms_per_step']*1e3,2), 'us/iter; sweep', round(d['roofline']['avg_launch_ms']*1e3,2))"
  done
done
