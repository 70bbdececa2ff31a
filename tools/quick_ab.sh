#!/bin/bash
# Quick GPU check of a kernel change: full GPU tests, bench at 500k / 62.5k, one SQ PMC pass
# of the 500k sweep.  Usage: tools/quick_ab.sh TAG
TAG=$1
mkdir -p gpurun_out/$TAG
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread \
  > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/pytest.log; ok $rc || exit $rc
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-binning --no-c5 --no-per-species --no-chemistry"
for n in 500000 62500; do
  timeout -k 10 200 $B --n-lam $n > gpurun_out/$TAG/bench_$n.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_$n.json'));print($n, 'ms/step %.4f'%d['ms_per_step'], 'sweep %.4f'%d['roofline']['avg_launch_ms'], d['sweep_path'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$TAG/pmc_sq -o run -- $B --steps 10 --warmup 1 --rad-eq-max 1 > gpurun_out/$TAG/pmc_sq.log 2>&1 || exit $?
python3 tools/pmc_valu.py gpurun_out/$TAG/pmc_sq gpurun_out/$TAG/valu.json
