#!/bin/bash
# Same-box bisect of the round-3 headline loss: bench.py's headline (the later legs off) for the
# round-2 tree, every round-3 commit that touched the kernels (built under abtree/<sha>) and
# HEAD, interleaved, $2 rounds.  One line per run: tree, updates/s, ms per T-P iteration, sweep
# event ms.
set -e -o pipefail
O=gpurun_out/${1:-r04bisect}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species"
TREES="r02 e9071f3 c1c6ad3 549be36 4ae958a 8e7b94c 186dd3d f0602e0 ad8346d 83fa468 HEAD"
for rep in $(seq 1 ${2:-3}); do
  for t in $TREES; do
    if [ $t = HEAD ]; then d=.; else d=abtree/$t; fi
    (cd $d && timeout -k 10 120 python3 bench.py $B) > $O/${t}_$rep.json 2> $O/${t}_$rep.err
    python3 -c "import json; d=json.load(open('$O/${t}_$rep.json')); print('$t', $rep, '%.4e' % d['value'], '%.4f' % d['ms_per_step'], '%.4f' % d['roofline']['avg_launch_ms'], flush=True)" | tee -a $O/summary.txt
  done
done
