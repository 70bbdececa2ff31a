#!/bin/bash
# Lanes-per-wavelength sweep: bench.py headline path at several λ slice sizes with Q forced
# to 1, 2 and 4 (FREI_GROUP_Q); one JSON line per run into gpurun_out/q_sweep.jsonl.
set -e
mkdir -p gpurun_out
out=gpurun_out/q_sweep.jsonl
: > $out
for lam in 250000 164000 125000 94000 62500 47000 31250; do
  for q in 1 2 4; do
    line=$(FREI_GROUP_Q=$q timeout -k 10 90 python bench.py --n-lam $lam --steps 30 --warmup 3 \
           --no-cpu-baseline --no-binning --no-c5 2>/dev/null)
    python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'n_lam':$lam,'q':$q,'ms_per_step':d['ms_per_step'],'sweep_ms':d['roofline']['avg_launch_ms']}))" "$line" | tee -a $out
  done
done
