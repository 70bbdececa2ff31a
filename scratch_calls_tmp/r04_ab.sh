#!/bin/bash
# Round-4 headline A/B on one box: the round-2 tree (8a7262a, built in abtree/r02) against HEAD,
# alternating, three bench runs each (headline only: the later legs do not touch it); then each
# tree's bench under a rocprofv3 kernel trace (the timed window's kernels and gaps,
# tools/window_gaps.py), and the in-kernel shader clock over the bench's window and after a soak
# (FREI_TRACE build, tools/clock_probe.py).
set -e -o pipefail
O=gpurun_out/${1:-r04ab}
mkdir -p $O
B="--no-cpu-baseline --no-binning --no-c5 --no-chemistry --no-per-species"
R=$GRAFT_REPO_ROOT
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py $B > $O/head_$i.json 2> $O/head_$i.err
  (cd abtree/r02 && timeout -k 10 150 python3 bench.py $B) > $O/r02_$i.json 2> $O/r02_$i.err
  python3 -c "import json; [print(t, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms']) for t in ('head_$i','r02_$i') for d in [json.load(open('$O/'+t+'.json'))]]"
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_head -o run -- python3 bench.py $B > $O/head_rocprof.json 2> $O/head_rocprof.err
(cd abtree/r02 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r02 -o run -- python3 bench.py $B) > $O/r02_rocprof.json 2> $O/r02_rocprof.err
python3 tools/window_gaps.py $O/prof_head/run_kernel_trace.csv > $O/window_head.txt
python3 tools/window_gaps.py $O/prof_r02/run_kernel_trace.csv > $O/window_r02.txt
cat $O/window_head.txt $O/window_r02.txt
FREI_HIP_LIB=abtree/trace.so timeout -k 10 200 python3 tools/clock_probe.py > $O/clock.txt 2> $O/clock.err
cat $O/clock.txt
