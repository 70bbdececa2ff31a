#!/bin/bash
# GPU check of the hipGraph replay: the whole GPU suite, then bench at 500k and 62.5k with
# graphs on / off (interleaved twice).  Outputs under gpurun_out/graph.
O=gpurun_out/graph
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 40 --warmup 8 --rad-eq-max 1 --no-cpu-baseline --no-binning --no-c5 --no-per-species --no-chemistry"
for rep in 1 2; do
for n in 500000 62500; do
  for g in 1 0; do
    FREI_GRAPH=$g timeout -k 10 200 $B --n-lam $n > $O/bench_${n}_g${g}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$O/bench_${n}_g${g}_$rep.json'));print($n, 'graph $g', 'ms/step %.4f'%d['ms_per_step'], 'value %.4g'%d['value'])"
  done
done
done
