#!/bin/bash
# One-lane sweep prefetch depth (steps in flight, FREI_PREFETCH_DEPTH = 1, 2, 4) at the
# one-lane slice sizes; 2 interleaved reps; one JSON line per run into gpurun_out/depth_sweep.jsonl.
set -e
mkdir -p gpurun_out
out=gpurun_out/depth_sweep.jsonl
: > $out
for rep in 1 2; do for lam in 500000 250000 125000; do
  for dep in 1 2 4; do
    line=$(FREI_PREFETCH_DEPTH=$dep timeout -k 10 90 python bench.py --n-lam $lam --steps 30 --warmup 3 \
           --no-cpu-baseline --no-binning --no-c5 2>/dev/null)
    python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'n_lam':$lam,'depth':$dep,'rep':$rep,'ms_per_step':d['ms_per_step'],'sweep_ms':d['roofline']['avg_launch_ms']}))" "$line" | tee -a $out
  done
done; done
