#!/bin/bash
# GPU check of the fused reduce + update: its bit-identity test, the multi-rank and RCCL
# tests, then bench at 500k and 62.5k (P2P forced on one rank) fused vs two kernels, and the
# 62.5k timelines.  Outputs under gpurun_out/fused.
O=gpurun_out/fused
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_fused_update.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py \
  > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 20 --warmup 5 --rad-eq-max 1 --no-cpu-baseline --no-binning --no-c5 --no-per-species --no-chemistry"
for n in 500000 62500; do
  for f in 1 0; do
    FREI_FUSED_UPDATE=$f timeout -k 10 200 $B --n-lam $n --force-comm > $O/bench_${n}_f$f.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$O/bench_${n}_f$f.json'));print($n, 'fused $f', 'ms/step %.4f'%d['ms_per_step'], 'sweep %.4f'%d['roofline']['avg_launch_ms'], d.get('exchange'))"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 1 0; do
  FREI_FUSED_UPDATE=$f timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof_f$f -o run -- $B --n-lam 62500 --force-comm > $O/bench_under_rocprof_f$f.json 2>/dev/null || exit $?
  python3 tools/timeline.py $O/prof_f$f/run_kernel_trace.csv | tee $O/timeline_n62500_f$f.txt
done
