# Round-2 measurement on one MI355X: PMC traffic + VALU passes of the contracted (headline) and
# per-species sweeps, the bench line, the rocprofv3 kernel-trace stats of the same command, the
# slice sizes of the 2/4/8-GPU runs and the 62.5k timeline with the one-rank P2P exchange.
# Outputs under gpurun_out/final2.
set -e
O=gpurun_out/final2
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
python3 tools/pmc_traffic.py $O/pmc_fetch_1 $O/pmc_write_1 profiles/traffic_sweep.json
python3 tools/pmc_valu.py $O/pmc_sq_1 profiles/valu_sweep.json
python3 tools/pmc_traffic.py $O/pmc_fetch_0 $O/pmc_write_0 profiles/traffic_sweep_per_species.json --contracted=0
python3 tools/pmc_valu.py $O/pmc_sq_0 profiles/valu_sweep_per_species.json
cp profiles/traffic_sweep*.json profiles/valu_sweep*.json $O/
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
for n in 250000 125000 62500; do
  timeout -k 10 120 python3 bench.py --n-lam $n --steps 20 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry > $O/bench_n$n.json 2>/dev/null
  timeout -k 10 120 python3 bench.py --n-lam $n --steps 20 --no-binning --no-cpu-baseline --no-c5 --no-per-species --force-comm > $O/bench_n${n}_p2p.json 2>/dev/null
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof_n62500 -o run -- python3 bench.py --n-lam 62500 --steps 20 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 --no-per-species --force-comm > $O/bench_n62500_under_rocprof.json 2>/dev/null
python3 tools/timeline.py $O/prof_n62500/run_kernel_trace.csv > $O/timeline_n62500.txt
python3 tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline_n500000.txt
