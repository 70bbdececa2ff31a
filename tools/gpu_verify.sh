#!/bin/bash
# GPU suite, smoke and the default bench line on the current tree.  gpurun_out/verify.
set -o pipefail
O=gpurun_out/verify
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['sweep_path']['setup_ms'], d['c5_batched']['rad_eq']['iterations_max'], d['c5_batched']['rad_eq']['converged_rank0'])"
