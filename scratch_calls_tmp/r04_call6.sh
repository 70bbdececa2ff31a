#!/bin/bash
# Round-4 GPU call: the whole GPU suite on the lean build (every failure listed, not only the
# first), with the parity log, then the default bench line.
set -o pipefail
O=gpurun_out/${1:-r04c6}
mkdir -p $O
FREI_PARITY_JSON=$O/parity.json timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail 25 --timeout 700 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -30; tail -2 $O/pytest.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['rad_eq']['iterations'], d['c5_batched']['updates_per_s'])"
