#!/bin/bash
# Trainer-config parity evidence (profiles/trajectory_r18_b32.md): the per-step trajectory diff at lr 0.05 (with the
# SGD-update / shadow checks), then the 3-path seed sweep. Usage (GPU box): bash scripts/runs/parity_sweep.sh [outdir] [seeds]
set -o pipefail
O=${1:-gpurun_out/parity}; SEEDS=${2:-0-5}
mkdir -p $O
BASE="--arch resnet18 --image-size 64 --data synthetic --synthetic-task colour --num-classes 10 --synthetic-val-size 1024 --log-interval 10 --warmup-epochs 0.5"
timeout -k 10 300 python -u scripts/trajectory_diff.py --out $O/traj_lr005_b32.jsonl -- $BASE --batch-size 32 --synthetic-train-size 4800 --lr 0.05 --epochs 2 > $O/traj_lr005_b32.log 2>&1 || exit 1
timeout -k 10 1500 python -u scripts/seed_sweep.py --seeds $SEEDS --out $O/sweep_lr005 -- --lr 0.05 > $O/sweep_lr005.log 2>&1 || exit 1
