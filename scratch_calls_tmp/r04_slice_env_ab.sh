#!/bin/bash
# 8-GPU slice: producer/consumer sweep with its default options vs records formed in the sweep
# (FREI_REC_SWEEP=1) and vs producers two phases ahead (FREI_PIPE_PF=2), one box, interleaved.
set -o pipefail
O=gpurun_out/${1:-r04slenv}
mkdir -p $O
B="--no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --steps 40 --warmup 5 --force-comm --lam-slice 0:62500"
for rep in 1 2 3; do
  for t in auto rec pf2; do
    case $t in
      auto) E="FREI_X=0";;
      rec) E="FREI_REC_SWEEP=1";;
      pf2) E="FREI_PIPE_PF=2";;
    esac
    env $E timeout -k 10 120 python3 bench.py $B > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_$rep.json')); print('$t', $rep, 'slice0 %.2f us per T-P iteration' % (a['ms_per_step']*1e3), flush=True)" | tee -a $O/summary.txt
  done
done
