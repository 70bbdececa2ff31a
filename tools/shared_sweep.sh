#!/bin/bash
# LDS step-table threshold sweep: bench.py headline path at several λ slice sizes with
# FREI_SHARED_MAX_BLOCKS = 0 (step table read from global memory) or 4096 (always in LDS);
# one JSON line per run into gpurun_out/shared_sweep.jsonl.
set -e
mkdir -p gpurun_out
out=gpurun_out/shared_sweep.jsonl
: > $out
for rep in 1 2 3; do for lam in ${LAMS:-500000 350000 250000 164000}; do
  for m in 0 4096; do
    line=$(FREI_SHARED_MAX_BLOCKS=$m timeout -k 10 90 python bench.py --n-lam $lam --steps 30 --warmup 3 \
           --no-cpu-baseline --no-binning --no-c5 2>/dev/null)
    python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'n_lam':$lam,'shared_max_blocks':$m,'rep':$rep,'ms_per_step':d['ms_per_step'],'sweep_ms':d['roofline']['avg_launch_ms']}))" "$line" | tee -a $out
  done
done; done
