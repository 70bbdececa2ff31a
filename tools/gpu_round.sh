#!/bin/bash
# One GPU-box session: GPU tests, then (unless a step faulted or timed out) bench.py.
# Usage: tools/gpu_round.sh TAG [pytest-args...]
# Exit statuses 0/1 (tests passed/failed) continue; anything else (timeout 124/137, abort
# 134, segfault 139, ...) stops the script so nothing more touches the GPU.
TAG=$1; shift
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread "$@" \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
ok $rc || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json \
  2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_$TAG.json
exit $rc
