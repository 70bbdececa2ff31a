#!/bin/bash
# groups-ahead A/B of the grouped-lane sweep: bit-identity test with GA=4, then bench at
# 47k / 62.5k / 94k, GA 2 vs 4 interleaved.  Outputs under gpurun_out/ga.
O=gpurun_out/ga
mkdir -p $O
FREI_GROUP_AHEAD=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "grouped" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 30 --warmup 5 --rad-eq-max 1 --no-cpu-baseline --no-binning --no-c5 --no-per-species --no-chemistry"
for rep in 1 2; do
for n in 47000 62500 94000; do
  for ga in 2 4; do
    FREI_GROUP_AHEAD=$ga timeout -k 10 200 $B --n-lam $n > $O/bench_${n}_ga${ga}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$O/bench_${n}_ga${ga}_$rep.json'));print($n, 'GA $ga', 'ms/step %.4f'%d['ms_per_step'], 'sweep %.4f'%d['roofline']['avg_launch_ms'], d['sweep_path']['paired'], d['sweep_path']['quad'])"
  done
done
done
