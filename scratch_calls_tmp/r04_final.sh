#!/bin/bash
# Round-4 final verification on one MI355X: the whole GPU suite with the parity log (provenance
# from .tree_stamp), smoke(), the driver's bench command, and the same bench under rocprofv3
# (kernel trace + stats; the timed window via tools/window_gaps.py).  Each GPU step has its own
# time limit; a failure ends the script.
set -e -o pipefail
O=gpurun_out/${1:-r04final}
mkdir -p $O
R=$GRAFT_REPO_ROOT
FREI_PARITY_JSON=$O/parity.json timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 700 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['rad_eq']['iterations'], d['cpu_baseline']['value'], d['c5_batched']['k7_roofline']['frac'])"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv > $O/trace_summary.txt 2>&1 || true
python3 tools/window_gaps.py --warmup 5 $O/prof/run_kernel_trace.csv > $O/window.txt 2>&1 || true
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
cat $O/window.txt
