#!/bin/bash
# Round-2 final refresh (after the producer/consumer sweep) on one MI355X: GPU tests, smoke, the
# bench line, the same bench under rocprofv3 (kernel trace + stats), PMC traffic + VALU passes of
# the contracted and per-species sweeps, the 2/4/8-GPU slice benches (with and without the
# one-rank P2P exchange), the per-sweep timelines, and the driver's N=2 and N=8 commands rehearsed
# with the ranks sharing this GPU over P2P.  Outputs under gpurun_out/final4; every GPU step has its
# own time limit and a failure ends the script.
set -e -o pipefail
O=gpurun_out/final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -3 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv > $O/trace_summary.txt 2>&1 || true
python3 tools/timeline.py $O/prof/run_kernel_trace.csv 500224 > $O/timeline_n500000.txt
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
for n in 250000 125000 62500; do
  timeout -k 10 120 python3 bench.py --n-lam $n --steps 20 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry > $O/bench_n$n.json 2>/dev/null
  timeout -k 10 120 python3 bench.py --n-lam $n --steps 20 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --force-comm > $O/bench_n${n}_p2p.json 2>/dev/null
  python3 -c "import json; a=json.load(open('$O/bench_n$n.json')); b=json.load(open('$O/bench_n${n}_p2p.json')); print($n, a['ms_per_step'], b['ms_per_step'], b['sweep_path'].get('pipe'))"
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof_n62500 -o run -- python3 bench.py --n-lam 62500 --steps 20 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --force-comm > $O/bench_n62500_under_rocprof.json 2>/dev/null
python3 tools/timeline.py $O/prof_n62500/run_kernel_trace.csv > $O/timeline_n62500_p2p.txt
cat $O/timeline_n62500_p2p.txt
MASTER_ADDR=127.0.0.1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-binning > $O/rehearsal_n2_p2p.json 2> $O/rehearsal_n2_p2p.err
MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --steps 10 --warmup 2 --no-cpu-baseline --no-binning > $O/rehearsal_n8_p2p.json 2> $O/rehearsal_n8_p2p.err
python3 -c "import json; [print(f, d['n_gpus'], d['ms_per_step'], d['rad_eq']['iterations'], d['config']['parallelism']) for f in ('n2','n8') for d in [json.load(open('$O/rehearsal_'+f+'_p2p.json'))]]"
