#!/bin/bash
# Where the producer/consumer sweep's longer launch gaps come from (62.5k slice, separate
# launches): pipe NC = 4 / 2, grouped-lane 4-wave blocks with and without a 150 KiB LDS floor
# (one block per CU, the pipe's LDS footprint).
set -e -o pipefail
O=gpurun_out/${1:-gap}
mkdir -p $O
T="timeout -k 10 120 python3 tools/trace_probe.py --n-lam 62500"
export FREI_HIP_LIB=abv/trace.so FREI_CHAIN=0
for cfg in "pipe4 FREI_PIPE=4" "pipe2 FREI_PIPE=2" "grp FREI_PIPE=0" "grp_lds150 FREI_PIPE=0 FREI_SWEEP_LDS_KB=150" "grp8_lds150 FREI_PIPE=0 FREI_GROUP_WAVES=8 FREI_SWEEP_LDS_KB=150"; do
  set -- $cfg
  tag=$1; shift
  env "$@" $T 2>/dev/null > $O/$tag.txt; echo "== $tag"; grep -A3 "kind" $O/$tag.txt | head -3; grep half $O/$tag.txt
done
