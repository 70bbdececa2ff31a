#!/bin/bash
# Forced one-rank P2P exchange at 125k/250k: current library vs the builds before the race fix and
# before in-sweep records (FREI_HIP_LIB), alternated; then the 8-rank shared-GPU rehearsal.
# gpurun_out/p2ps.
set -o pipefail
O=gpurun_out/p2ps
mkdir -p $O
B="python3 bench.py --steps 20 --no-binning --no-cpu-baseline --no-c5 --no-per-species --no-chemistry --rad-eq-max 1"
for r in 1 2; do
  for n in 125000 250000; do
    for v in cur prefix prerec; do
      lib=frei_amd/libfrei_hip.so; [ $v = prefix ] && lib=tools/ab_prefix.so; [ $v = prerec ] && lib=tools/ab_prerec.so
      FREI_HIP_LIB=$lib timeout -k 10 120 $B --n-lam $n --force-comm > $O/${v}_${n}_${r}.json 2>/dev/null || exit $?
      python3 -c "import json; d=json.load(open('$O/${v}_${n}_${r}.json')); print('$v', $n, $r, round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['exchange']['avg_ms'])"
    done
    FREI_REC_SWEEP=0 timeout -k 10 120 $B --n-lam $n --force-comm > $O/rec0_${n}_${r}.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$O/rec0_${n}_${r}.json')); print('cur_rec0', $n, $r, round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['exchange']['avg_ms'])"
  done
done
MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --steps 10 --warmup 2 --no-cpu-baseline --no-binning > $O/rehearsal_n8_p2p.json 2> $O/rehearsal_n8_p2p.err || exit $?
python3 -c "import json; d=json.load(open('$O/rehearsal_n8_p2p.json')); print('n8', d['ms_per_step'], d['rad_eq']['iterations'], d['sweep_path'].get('pipe'))"
