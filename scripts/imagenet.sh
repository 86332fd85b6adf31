#!/bin/bash
# Slurm job for MI355X nodes: one task per GPU, RCCL over xGMI inside a node.
#
# Counterpart of the reference's imagenet.sh (8 nodes x 2 GPUs, NCCL over TCP
# with P2P and IB disabled). Differences, on purpose:
#  * 8 tasks per node (one per MI355X), one node by default;
#  * NO NCCL_P2P_DISABLE / NCCL_IB_DISABLE / NCCL_LL_THRESHOLD: RCCL must use
#    the 7 point-to-point xGMI links (and RDMA between nodes);
#  * enough CPUs per task for the JPEG decode workers (the reference squeezed
#    10 workers into 1 CPU per task);
#  * HSA_ENABLE_IPC_MODE_LEGACY=0 (dmabuf IPC) for RCCL peer memory.
#
#SBATCH --job-name=imagenet_mi355x
#SBATCH --nodes=1
#SBATCH --ntasks-per-node=8
#SBATCH --gres=gpu:8
#SBATCH --cpus-per-task=12
#SBATCH --exclusive
#SBATCH --time=24:00:00
#SBATCH --output=imagenet_SGD.out
#SBATCH --error=imagenet_SGD.err

set -x
cd "${SLURM_SUBMIT_DIR:-.}"

export HSA_ENABLE_IPC_MODE_LEGACY=0
export OMP_NUM_THREADS=${SLURM_CPUS_PER_TASK:-8}

srun python ./imagenet.py --backend=nccl --launcher slurm \
    --arch "${ARCH:-resnet50}" --image-size "${IMAGE_SIZE:-224}" --batch-size "${BATCH:-256}" \
    --workers "${WORKERS:-10}" "$@"
