#!/bin/bash
# P2P push without the system-scope release fence: GPU suite (2/4/8-rank P2P tests), then the
# forced one-rank exchange at the 2/4/8-GPU slices, fence vs no fence, alternated.  gpurun_out/p2pf.
set -o pipefail
O=gpurun_out/p2pf
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 30 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1"
for r in 1 2; do
  for n in 250000 125000 62500; do
    for v in nofence fence; do
      lib=frei_amd/libfrei_hip.so; [ $v = fence ] && lib=tools/ab_fence.so
      FREI_HIP_LIB=$lib timeout -k 10 120 $B --n-lam $n --force-comm > $O/${v}_${n}_${r}.json 2>/dev/null || exit $?
      python3 -c "import json; d=json.load(open('$O/${v}_${n}_${r}.json')); print('$v $n $r', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['exchange']['avg_ms'])"
    done
  done
done
MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-binning > $O/rehearsal_n2_p2p.json 2> $O/rehearsal_n2_p2p.err || exit $?
python3 -c "import json; d=json.load(open('$O/rehearsal_n2_p2p.json')); print('n2', d['ms_per_step'], d['rad_eq']['iterations'])"
