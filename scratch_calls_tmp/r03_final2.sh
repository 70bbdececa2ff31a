#!/bin/bash
# Final tree: math bit-identity checks, GPU tests, smoke, bench, bench under rocprofv3.
set -e -o pipefail
O=gpurun_out/${1:-final2}
mkdir -p $O
timeout -k 10 300 ./tools/mathcheck > $O/mathcheck.txt 2>&1; cat $O/mathcheck.txt
bash tools/calls/r03_verify.sh ${1:-final2}
