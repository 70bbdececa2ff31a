#!/bin/bash
# Round-3 verification on one MI355X: GPU tests, smoke, the default bench line and the same bench
# under rocprofv3 (kernel trace + stats).  Outputs under gpurun_out/$1; every GPU step has its own
# time limit and a failure ends the script.
set -e -o pipefail
O=gpurun_out/${1:-verify}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -3 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('c5_batched',{}).get('k7_roofline'))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv > $O/trace_summary.txt 2>&1 || true
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
