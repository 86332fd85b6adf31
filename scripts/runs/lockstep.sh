#!/bin/bash
# Lockstep trajectories (HIP vs PyTorch fp32 vs PyTorch bf16 autocast from one start, same batches / lr / SGD):
# how fast each departs from the fp32 trajectory. Usage (GPU box): bash scripts/runs/lockstep.sh [outdir] [seeds...]
set -o pipefail
O=${1:-gpurun_out/lockstep}; shift || true
SEEDS=${@:-0 2 5}
mkdir -p $O
BASE="--arch resnet18 --image-size 64 --data synthetic --synthetic-task colour --num-classes 10 --synthetic-val-size 1024 --log-interval 10 --warmup-epochs 0.5 --batch-size 32 --synthetic-train-size 4800 --lr 0.05 --epochs 2"
for s in $SEEDS; do
  timeout -k 10 300 python -u scripts/trajectory_diff.py --lockstep --out $O/lock_s$s.jsonl -- $BASE --seed $s > $O/lock_s$s.log 2>&1 || exit 1
done
