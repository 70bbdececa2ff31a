#!/bin/bash
# After the stream-ordering fix: GPU suite, C5 after a C3 context (twice), and the bench's
# C5-only order that showed the anomaly.  gpurun_out/race.
set -o pipefail
O=gpurun_out/race
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 tools/c5_determinism.py 100000 -1.0 0 afterc3 > $O/after$i.txt 2>&1 || exit $?
  echo "afterc3 $i: $(tail -1 $O/after$i.txt)"
done
bash tools/c5_repro.sh
