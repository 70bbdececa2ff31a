#!/bin/bash
# Small-slice sweep check: grouped-lane bit-identity tests, bench at 62.5k / 125k (sweep
# HIP-event time), one SQ PMC pass at 62.5k (VALU per update).  Outputs under gpurun_out/ss.
O=gpurun_out/ss
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "grouped or contraction or c1" tests/test_gpu_fused_update.py \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 30 --warmup 5 --rad-eq-max 1 --no-cpu-baseline --no-binning --no-c5 --no-per-species --no-chemistry"
for rep in 1 2; do
for n in 62500 125000; do
  timeout -k 10 200 $B --n-lam $n > $O/bench_${n}_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('$O/bench_${n}_$rep.json'));print($n, 'ms/step %.4f'%d['ms_per_step'], 'sweep %.4f'%d['roofline']['avg_launch_ms'], d['sweep_path']['paired'], d['sweep_path']['quad'])"
done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_sq -o run -- $B --n-lam 62500 --steps 10 > $O/pmc_sq.log 2>&1 || exit $?
python3 tools/pmc_valu.py $O/pmc_sq $O/valu_62500.json --n-lam=62500 && cat $O/valu_62500.json
