#!/bin/bash
# Paired trailing-update launches at the 8-GPU slice: the trailing-update GPU tests, then slice
# 5/8 of the 500k grid (one-rank P2P and local) with FREI_TAIL_PAIR=1 / 0 interleaved.  A wait
# that gives up fails within FREI_P2P_TIMEOUT_S = 3.
set -o pipefail
O=gpurun_out/${1:-pair_ab}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tail.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="python3 bench.py --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --no-provider --rad-eq-max 1 --steps 40 --warmup 5"
export FREI_P2P_TIMEOUT_S=3
for rep in 1 2; do
  for comm in p2p local; do
    F=""; [ $comm = p2p ] && F="--force-comm"
    for v in 1 0; do
      f=$O/s5_${comm}_pair${v}_$rep
      if FREI_TAIL_PAIR=$v timeout -k 10 150 $B $F --lam-slice 312500:375000 > $f.json 2> $f.err; then
        python3 -c "import json; d=json.load(open('$f.json')); print('slice 5/8 $comm pair $v rep $rep', round(d['ms_per_step']*1e3,2), 'us per T-P iteration, path', d['sweep_path'].get('tail_pair'))"
      else
        echo "slice 5/8 $comm pair $v rep $rep FAILED: $(tail -1 $f.err)"; exit 1
      fi
    done
  done
done
