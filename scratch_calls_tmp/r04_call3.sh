#!/bin/bash
# Round-4 GPU call: (1) the headline A/B around the regressing commit 186dd3d — its parent
# 8e7b94c, 186dd3d, 8e7b94c with 186dd3d's three extra small context allocations (abtree/e2), and
# HEAD — interleaved 3 rounds, plus rocprofv3 kernel traces of 8e7b94c's and 186dd3d's benches;
# (2) the GPU tests touched this round.  A test failure (rc 1) does not stop later steps; a
# timeout, abort or signal (rc >= 124) ends the script.
set -o pipefail
O=gpurun_out/${1:-r04c3}
mkdir -p $O
R=$GRAFT_REPO_ROOT
step() {  # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species"
for rep in 1 2 3; do
  for t in 8e7b94c e2 186dd3d HEAD; do
    if [ $t = HEAD ]; then d=.; else d=abtree/$t; fi
    (cd $d && timeout -k 10 120 python3 bench.py $B) > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; d=json.load(open('$O/${t}_$rep.json')); print('$t', $rep, '%.4e' % d['value'], '%.4f' % d['ms_per_step'], '%.4f' % d['roofline']['avg_launch_ms'], flush=True)" | tee -a $O/summary.txt
  done
done
export TMPDIR=/tmp
for t in 8e7b94c 186dd3d; do
  (cd abtree/$t && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof_$t -o run -- python3 bench.py $B) > $O/${t}_rocprof.json 2> $O/${t}_rocprof.err || { echo "rocprof $t failed"; exit 3; }
  python3 tools/window_gaps.py $O/prof_$t/run_kernel_trace.csv > $O/window_$t.txt 2>&1; cat $O/window_$t.txt
done
P="python -u -m pytest -x -v --timeout 700 --timeout-method thread"
step mr_default 300 $P tests/test_gpu_multirank.py
FREI_CHAIN_SHARED=1 step mr_chain_shared 300 $P tests/test_gpu_multirank.py -k "p2p"
step provider 300 $P tests/test_gpu_chemistry_provider.py
step boundary 300 $P tests/test_gpu_boundary.py
step radeq 900 $P tests/test_gpu_radeq_fullsize.py
grep -h -E "passed|failed" $O/*.log | tail -8
