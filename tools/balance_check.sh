#!/bin/bash
# Cost-balanced slicing rehearsed with ranks sharing this GPU (--balance forces the calibration,
# which is otherwise skipped when ranks share a GPU), N = 2 and 4, P2P; then the GPU tests of the
# multi-rank and chain paths.
set -e -o pipefail
O=gpurun_out/${1:-bal}
mkdir -p $O
for n in 2 4; do
  MASTER_ADDR=127.0.0.1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2954$n bench.py --gpus $n --steps 10 --warmup 2 --no-cpu-baseline --no-binning --no-c5 --no-per-species --no-chemistry --balance > $O/bal_n$n.json 2> $O/bal_n$n.err
  python3 -c "import json; d=json.load(open('$O/bal_n$n.json')); print($n, d['ms_per_step'], d['rad_eq']['iterations'], d['config']['slicing'])"
done
