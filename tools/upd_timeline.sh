#!/bin/bash
# Fused-update duration by ablation (diagnostic builds; their results are wrong by design,
# timing only): rocprofv3 kernel trace of bench.py at N lambda (one-lane sweep at 500k) for the
# current build and abv/upd_{nosum,nodt,empty}.so, then the per-half medians (tools/timeline.py).
set -e -o pipefail
O=${1:-gpurun_out/updt}
N=${2:-500000}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --n-lam $N --steps 20 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry"
for v in full nosum nodt empty; do
  if [ $v = full ]; then unset FREI_HIP_LIB; else export FREI_HIP_LIB=abv/upd_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- $B > $O/$v.json 2>/dev/null
  echo "== $v"; python3 tools/timeline.py $O/$v/run_kernel_trace.csv
done
unset FREI_HIP_LIB
