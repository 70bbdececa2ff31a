#!/bin/bash
# Small-slice diagnostics: memory-only one-lane build vs the full one, and the sweep time at
# 30/60/120 layers (fixed per-launch overhead vs per-step cost).  Outputs under gpurun_out/probe.
set -o pipefail
O=gpurun_out/probe
mkdir -p $O
L=frei_amd/libfrei_hip.so
timeout -k 10 200 python -u tools/ab_sweep.py --n-lam=62500 --rounds=7 --iters=8 \
  one=$L@FREI_GROUP_Q=1,FREI_PIPE=0 mem=tools/ab_memonly.so@FREI_GROUP_Q=1,FREI_PIPE=0 \
  grp=$L@FREI_PIPE=0 p4=$L@FREI_PIPE=4,FREI_PIPE_PF=1 > $O/ab_mem.txt 2>&1 || exit $?
cat $O/ab_mem.txt
for nl in 30 60 120; do
  for v in 0 4; do
    FREI_PIPE=$v FREI_PIPE_PF=1 timeout -k 10 120 python3 bench.py --n-lam 62500 --n-layers $nl --steps 20 --rad-eq-max 1 \
      --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry > $O/b_${nl}_$v.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$O/b_${nl}_$v.json')); print($nl, $v, d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
