#!/bin/bash
# Whole GPU suite, then the default bench line (C5 leg with the two-wavelength batched sweep).
set -o pipefail
O=gpurun_out/${1:-r04c12}
mkdir -p $O
FREI_PARITY_JSON=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 700 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -1 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['c5_batched']; print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], 'C5', c['updates_per_s'], c['ms_per_step'], c['rad_eq'])"
