#!/bin/bash
# Bit-identity tests with the two-wavelength form, then the in-kernel trace of a 500k half
# iteration (FREI_TRACE build): sweep_pair blocks and the fused update's phases.
set -o pipefail
O=gpurun_out/${1:-r04c11}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_update.py tests/test_gpu_lam2.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head; tail -1 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
FREI_HIP_LIB=ablib/trace.so timeout -k 10 200 python3 tools/trace_probe.py --n-lam 500000 --iters 20 --blocks > $O/trace500.txt 2>&1
head -12 $O/trace500.txt
