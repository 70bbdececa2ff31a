#!/bin/bash
# Round-6 final verification on one MI355X (outputs under gpurun_out/r06final, or gpurun_out/$1):
#   the GPU suite with the parity log, smoke(), the driver's bench line, rocprofv3 kernel-trace
#   stats of the same bench command, and the PMC passes (HBM traffic, VALU) of the headline
#   sweep and of the per-species sweep.  Every GPU step under its own time limit; stop at the
#   first failure.
set -o pipefail
O=gpurun_out/${1:-r06final}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -m tests.provenance > $O/tree_hash.txt 2>&1
FREI_PARITY_JSON=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 11
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 12
tail -1 $O/smoke.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 13
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['rad_eq']['iters_per_s_incl_setup'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err || exit 14
B="python3 bench.py --steps 10 --warmup 1 --rad-eq-max 1 --no-cpu-baseline --no-binning --no-c5 --no-provider --no-chemistry"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 || exit 15
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 || exit 16
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -o run -- $B > $O/pmc_sq.log 2>&1 || exit 17
echo done
