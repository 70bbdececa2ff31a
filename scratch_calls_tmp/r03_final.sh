#!/bin/bash
# Round-3 verification + projection: GPU tests, smoke, bench, bench under rocprofv3, PMC passes,
# the per-rank slice projection, and the driver's N=2 / N=8 commands rehearsed with ranks sharing
# this GPU.
set -e -o pipefail
O=gpurun_out/${1:-final}
bash tools/calls/r03_verify.sh ${1:-final}
bash tools/calls/r03_pmc.sh ${1:-final}_pmc
bash tools/projection.sh ${1:-final}_proj
MASTER_ADDR=127.0.0.1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-binning > $O/rehearsal_n2.json 2> $O/rehearsal_n2.err
MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --steps 10 --warmup 2 --no-cpu-baseline --no-binning > $O/rehearsal_n8.json 2> $O/rehearsal_n8.err
python3 -c "import json; [print(f, d['n_gpus'], d['ms_per_step'], d['rad_eq']['iterations'], d['config']['parallelism']) for f in ('n2','n8') for d in [json.load(open('$O/rehearsal_'+f+'.json'))]]"
