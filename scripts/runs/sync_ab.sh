#!/bin/bash
# Loss-spike frequency of the HIP trainer with / without CPU run-ahead and the weight-gradient side stream, against the
# fp32 oracle, over many seeds (2 epochs at lr 0.05). Usage: bash scripts/runs/sync_ab.sh [outdir] [seeds] [paths]
set -o pipefail
O=${1:-gpurun_out/sync_ab}; SEEDS=${2:-10-19}; PATHS=${3:-hip_bf16,hip_sync,hip_nowgs,torch_fp32}
mkdir -p $O
timeout -k 10 1150 python -u scripts/seed_sweep.py --seeds $SEEDS --paths $PATHS --out $O/sweep -- --lr 0.05 > $O/sweep.log 2>&1 || exit 1
