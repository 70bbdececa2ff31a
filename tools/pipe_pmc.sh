#!/bin/bash
# SQ stall/instruction passes of the small-slice sweep forms (62.5k lambda): grouped-lane vs
# producer/consumer.  Outputs under gpurun_out/ppmc.
set -o pipefail
O=gpurun_out/ppmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --n-lam 62500 --steps 10 --warmup 1 --rad-eq-max 1 --no-cpu-baseline --no-binning --no-c5 --no-per-species --no-chemistry"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
for v in 0 4; do
  export FREI_PIPE=$v
  timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/p1_$v -o run -- $B > $O/p1_$v.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $O/p2_$v -o run -- $B > $O/p2_$v.log 2>&1 || exit $?
  python3 tools/pmc_stall.py $O/p1_$v $O/p2_$v --n-lam=62500 | tee $O/stall_$v.txt
done
