#!/bin/bash
# C5 after a C3 context in the same process (device VA reuse), vs alone.  gpurun_out/c5va.
set -o pipefail
O=gpurun_out/c5va
mkdir -p $O
timeout -k 10 300 python3 tools/c5_determinism.py 100000 -1.0 0 afterc3 > $O/after1.txt 2>&1 || exit $?
cat $O/after1.txt
timeout -k 10 300 python3 tools/c5_determinism.py 100000 -1.0 0 afterc3 > $O/after2.txt 2>&1 || exit $?
cat $O/after2.txt
bash tools/c5_repro.sh
