#!/bin/bash
# Exchange fallback chain: 2 ranks sharing this GPU with P2P setup failing on every rank
# (FREI_FAULT_P2P=1): RCCL, or the host all-gather where RCCL cannot run; one JSON line.
set -o pipefail
O=gpurun_out/fb
mkdir -p $O
FREI_FAULT_P2P=1 MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --no-binning --no-per-species --no-chemistry > $O/fb.json 2> $O/fb.err || { tail -30 $O/fb.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/fb.json')); print(d['n_gpus'], d['ms_per_step'], d['rad_eq']['iterations'], d['exchange'])"
