#!/bin/bash
# Round-4 GPU call: the lean coefficient form (HEAD, FREI_LEAN=1) against the literal form
# (abtree/nolean.so, FREI_LEAN=0): interleaved headline benches, 3 rounds; the whole GPU suite on
# the lean build with the parity log; the PMC VALU pass of the contracted 500k sweep.
set -o pipefail
O=gpurun_out/${1:-r04c5}
mkdir -p $O
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species --steps 20 --warmup 5"
for rep in 1 2 3; do
  for t in lean nolean; do
    if [ $t = lean ]; then L=""; else L="FREI_HIP_LIB=abtree/nolean.so"; fi
    env $L timeout -k 10 120 python3 bench.py $B > $O/${t}_$rep.json 2> $O/${t}_$rep.err || { echo "bench $t failed"; exit 3; }
    python3 -c "import json; d=json.load(open('$O/${t}_$rep.json')); print('$t', $rep, '%.4e' % d['value'], '%.4f' % d['ms_per_step'], '%.4f' % d['roofline']['avg_launch_ms'], flush=True)" | tee -a $O/summary.txt
  done
done
FREI_PARITY_JSON=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
if [ $rc -ge 124 ]; then exit $rc; fi
export TMPDIR=/tmp
PB="python3 bench.py --steps 10 --warmup 1 --rad-eq-max 1 --no-cpu-baseline --no-binning --no-c5 --no-per-species --no-chemistry"
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $R/$O/pmc_sq_1 -o run -- $PB > $O/pmc_sq_1.log 2>&1 || { echo "pmc failed"; exit 3; }
python3 tools/pmc_valu.py $O/pmc_sq_1 $O/valu_sweep.json && cat $O/valu_sweep.json
