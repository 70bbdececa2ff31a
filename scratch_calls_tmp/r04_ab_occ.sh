#!/bin/bash
# A/B at 500k (interleaved, one box): the current build with its default load ring (two steps
# ahead), eight steps ahead (FREI_PREFETCH_STEPS=8), four steps per coefficient block
# (FREI_PREFETCH_DEPTH=4), and a build held to 96 VGPRs for 5 waves per SIMD (FREI_LB_WAVES=5).
set -o pipefail
O=gpurun_out/${1:-r04occ}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  for t in cur pf8 pd4 lb5; do
    case $t in
      cur) E="FREI_HIP_LIB=ablib/cur.so";;
      pf8) E="FREI_HIP_LIB=ablib/cur.so FREI_PREFETCH_STEPS=8";;
      pd4) E="FREI_HIP_LIB=ablib/cur.so FREI_PREFETCH_DEPTH=4";;
      lb5) E="FREI_HIP_LIB=ablib/lb5.so";;
    esac
    env $E timeout -k 10 120 python3 bench.py $B > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_$rep.json')); print('$t', $rep, '500k %.4f ms sweep %.2f us' % (a['ms_per_step'], a['roofline']['avg_launch_ms']*1e3), flush=True)" | tee -a $O/summary.txt
  done
done
