#!/bin/bash
# Kernel traces at 250k with and without the forced one-rank P2P exchange.  gpurun_out/p2pt.
set -o pipefail
O=gpurun_out/p2pt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 20 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1 --n-lam 250000"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/none -o run -- $B > $O/none.json 2>/dev/null || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/p2p -o run -- $B --force-comm > $O/p2p.json 2>/dev/null || exit $?
python3 tools/timeline.py $O/none/run_kernel_trace.csv 977 > $O/tl_none.txt; cat $O/tl_none.txt
python3 tools/timeline.py $O/p2p/run_kernel_trace.csv 977 > $O/tl_p2p.txt; cat $O/tl_p2p.txt
