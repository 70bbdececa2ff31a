# Round-end measurement on one MI355X: PMC traffic + VALU passes, the bench line, and the
# rocprofv3 kernel-trace stats of the same command.  Outputs under gpurun_out/final.
set -e
mkdir -p gpurun_out/final
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 10 --warmup 1 --rad-eq-max 1 --no-cpu-baseline --no-binning --no-c5"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/final/pmc_fetch -o run -- $B > gpurun_out/final/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/final/pmc_write -o run -- $B > gpurun_out/final/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/final/pmc_sq -o run -- $B > gpurun_out/final/pmc_sq.log 2>&1
python3 tools/pmc_traffic.py gpurun_out/final/pmc_fetch gpurun_out/final/pmc_write profiles/traffic_sweep.json
python3 tools/pmc_valu.py gpurun_out/final/pmc_sq profiles/valu_sweep.json
cp profiles/traffic_sweep.json profiles/valu_sweep.json gpurun_out/final/
timeout -k 10 400 python3 bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/final/bench_under_rocprof.json 2> gpurun_out/final/bench_under_rocprof.err
# per-GPU slice sizes of the 2/4/8-GPU runs on one GPU (sweep + fixed per-sweep costs)
for n in 250000 125000 62500; do
  timeout -k 10 120 python3 bench.py --n-lam $n --steps 20 --no-binning --no-cpu-baseline --no-c5 > gpurun_out/final/bench_n$n.json 2>/dev/null
done
# per-sweep timeline (kernel durations and gaps) at the 8-GPU slice size
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/final/prof_n62500 -o run -- python3 bench.py --n-lam 62500 --steps 20 --rad-eq-max 1 --no-binning --no-cpu-baseline --no-c5 > gpurun_out/final/bench_n62500_under_rocprof.json 2>/dev/null
python3 tools/timeline.py gpurun_out/final/prof_n62500/run_kernel_trace.csv > gpurun_out/final/timeline_n62500.txt
python3 tools/timeline.py gpurun_out/final/prof/run_kernel_trace.csv > gpurun_out/final/timeline_n500000.txt
