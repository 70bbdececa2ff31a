#!/bin/bash
# One-lane chained launches: the chain bit-identity tests, then the producer/consumer layout A/B
# (tools/pipe_rot_ab.sh), then alternating bench A/B of chain off / on at the 4- and 2-GPU slices
# and at 500k (LDS step records forced on with FREI_SHARED=1 above 640 blocks).
set -e -o pipefail
O=gpurun_out/${1:-chol}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash tools/pipe_rot_ab.sh ${1:-chol}_pipe
B="python3 bench.py --steps 30 --warmup 5 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry"
for r in 1 2; do
  for cfg in "125000 0 -1" "125000 1 -1" "250000 0 -1" "250000 0 1" "250000 1 1" "500000 0 -1" "500000 0 1" "500000 1 1"; do
    set -- $cfg
    FREI_CHAIN=$2 FREI_SHARED=$3 timeout -k 10 120 $B --n-lam $1 > $O/b_$1_$2_$3_$r.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/b_$1_$2_$3_$r.json')); print('n $1 chain $2 shared $3', $r, round(d['ms_per_step']*1e3,2), 'us/iter; sweep', round(d['roofline']['avg_launch_ms']*1e3,2))"
  done
done
