#!/bin/bash
# Round-4 GPU call: the headline after the check_comm fix (HEAD) against 8e7b94c, interleaved, 3
# rounds, HEAD's bench under a rocprofv3 kernel trace (timed window), then the provider and C5
# full-size tests.  A test failure (rc 1) does not stop later steps; rc >= 124 ends the script.
set -o pipefail
O=gpurun_out/${1:-r04c4}
mkdir -p $O
R=$GRAFT_REPO_ROOT
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  for t in 8e7b94c HEAD; do
    if [ $t = HEAD ]; then d=.; else d=abtree/$t; fi
    (cd $d && timeout -k 10 120 python3 bench.py $B) > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; d=json.load(open('$O/${t}_$rep.json')); print('$t', $rep, '%.4e' % d['value'], '%.4f' % d['ms_per_step'], '%.4f' % d['roofline']['avg_launch_ms'], flush=True)" | tee -a $O/summary.txt
  done
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof_HEAD -o run -- python3 bench.py $B > $O/HEAD_rocprof.json 2> $O/HEAD_rocprof.err || { echo "rocprof failed"; exit 3; }
python3 tools/window_gaps.py --warmup 5 $O/prof_HEAD/run_kernel_trace.csv > $O/window_HEAD.txt 2>&1; cat $O/window_HEAD.txt
P="python -u -m pytest -x -v --timeout 700 --timeout-method thread"
step provider 300 $P tests/test_gpu_chemistry_provider.py
step c5 600 $P tests/test_gpu_c5_fullsize.py
grep -h -E "passed|failed" $O/*.log | tail -4
