#!/bin/bash
# Seed sweep of the trainer-test schedule: lr 0.05 (half-epoch warmup) for 2 epochs, then the reference's step decay
# (x0.1, imagenet.py:154-162) for a third epoch, on the three paths. Usage: bash scripts/runs/decay_sweep.sh [outdir] [seeds]
set -o pipefail
O=${1:-gpurun_out/decay}; SEEDS=${2:-0-3}
mkdir -p $O
timeout -k 10 1100 python -u scripts/seed_sweep.py --seeds $SEEDS --out $O/sweep -- --lr 0.05 --epochs 3 --lr-step 2 > $O/sweep.log 2>&1 || exit 1
