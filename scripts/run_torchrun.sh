#!/bin/bash
# Single-node launch without Slurm: one rank per MI355X.
#   scripts/run_torchrun.sh 8 --arch resnet50 --image-size 224 --data synthetic
set -e
NGPU=${1:-8}
shift || true
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$(dirname "$0")/.."
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" \
    --master-addr 127.0.0.1 --master-port "${MASTER_PORT:-29500}" \
    imagenet.py --backend=nccl --launcher torchrun "$@"
