#!/bin/bash
# GPU tests, then the 62.5k-slice bench (auto sweep choice, P2P exchange forced on one rank)
# with a rocprof kernel trace for the per-sweep timeline.  Outputs under gpurun_out/pr.
set -o pipefail
O=gpurun_out/pr
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 62500 125000 250000; do
  timeout -k 10 120 python3 bench.py --n-lam $n --steps 20 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --force-comm > $O/bench_n${n}_p2p.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_n${n}_p2p.json')); print($n, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['sweep_path'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof_n62500 -o run -- python3 bench.py --n-lam 62500 --steps 20 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --force-comm > $O/bench_n62500_under_rocprof.json 2>/dev/null || exit $?
python3 tools/timeline.py $O/prof_n62500/run_kernel_trace.csv > $O/timeline_n62500.txt
cat $O/timeline_n62500.txt
