#!/bin/bash
# A/B: Planck from the transmission's exp (FREI_PLANCK_EXP, 20 VGPRs fewer: 5 waves per SIMD for
# the 500k sweep, 4 for the grouped-lane slice sweep) vs the previous build (ablib/ring.so), and
# the one-step coefficient block with loads two steps ahead (depth 1, prefetch 2); interleaved at
# 500k and at the 8-GPU slice.  Then the whole GPU suite on the new build.
set -o pipefail
O=gpurun_out/${1:-r04pexp}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  for t in updb prio head pexp ring d1pf2; do
    case $t in
      pexp) E="FREI_HIP_LIB=ablib/pexp.so";;
      head) E="FREI_HIP_LIB=ablib/head.so";;
      updb) E="FREI_HIP_LIB=ablib/updb.so";;
      prio) E="FREI_HIP_LIB=ablib/prio.so";;
      ring) E="FREI_HIP_LIB=ablib/ring.so";;
      d1pf2) E="FREI_HIP_LIB=ablib/updb.so FREI_PREFETCH_DEPTH=1 FREI_PREFETCH_STEPS=2";;
    esac
    env $E timeout -k 10 120 python3 bench.py $B > $O/${t}_500k_$rep.json 2> $O/${t}_500k_$rep.err || { echo "bench $t failed"; exit 3; }
    env $E timeout -k 10 120 python3 bench.py $B --rad-eq-max 1 --steps 40 --force-comm --lam-slice 0:62500 > $O/${t}_s0_$rep.json 2> /dev/null || { echo "bench slice $t failed"; exit 3; }
    python3 -c "import json; a=json.load(open('$O/${t}_500k_$rep.json')); b=json.load(open('$O/${t}_s0_$rep.json')); print('$t', $rep, '500k %.4f ms sweep %.2f us' % (a['ms_per_step'], a['roofline']['avg_launch_ms']*1e3), 'slice0 %.2f us' % (b['ms_per_step']*1e3), flush=True)" | tee -a $O/summary.txt
  done
done
bash tools/calls/r04_rounds.sh ${1:-r04pexp}/rounds
FREI_PARITY_JSON=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 700 --timeout-method thread > $O/pytest.log 2>&1
grep -E "FAILED" $O/pytest.log | head -20; tail -1 $O/pytest.log
