#!/bin/bash
# world_size-2 rehearsal of bench.py on ONE GPU with the gloo backend (RCCL needs 2 GPUs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp CZ_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dist2.log 2>&1
rc=$?; tail -3 gpurun_out/dist2.log; exit $rc
