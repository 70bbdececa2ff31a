#!/bin/bash
# PMC passes of the headline sweep (contracted, 1) and the per-species sweep (0): FETCH_SIZE,
# WRITE_SIZE and the SQ VALU counters, each its own run; summarised into profiles-style JSON.
set -e -o pipefail
O=gpurun_out/${1:-pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 10 --warmup 1 --rad-eq-max 1 --no-cpu-baseline --no-binning --no-c5 --no-per-species --no-chemistry"
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for mode in 1 0; do
  export FREI_PRECONTRACT=$mode
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$mode -o run -- $B > $O/pmc_fetch_$mode.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$mode -o run -- $B > $O/pmc_write_$mode.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_sq_$mode -o run -- $B > $O/pmc_sq_$mode.log 2>&1
done
unset FREI_PRECONTRACT
python3 tools/pmc_traffic.py $O/pmc_fetch_1 $O/pmc_write_1 $O/traffic_sweep.json
python3 tools/pmc_valu.py $O/pmc_sq_1 $O/valu_sweep.json
python3 tools/pmc_traffic.py $O/pmc_fetch_0 $O/pmc_write_0 $O/traffic_sweep_per_species.json --contracted=0
python3 tools/pmc_valu.py $O/pmc_sq_0 $O/valu_sweep_per_species.json
cat $O/traffic_sweep.json $O/valu_sweep.json | head -40
