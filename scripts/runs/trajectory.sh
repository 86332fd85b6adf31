#!/bin/bash
# Trajectory diffs of the HIP trainer vs PyTorch fp32 / bf16-autocast on the HIP weights
# (profiles/trajectory_r18_b32.md). Usage: bash scripts/runs/trajectory.sh [outdir]
set -e
O=${1:-gpurun_out/traj}
mkdir -p $O
BASE="--arch resnet18 --image-size 64 --data synthetic --synthetic-task colour --num-classes 10 --synthetic-val-size 1024 --log-interval 10 --warmup-epochs 0.5"
timeout -k 10 300 python -u scripts/trajectory_diff.py --out $O/lr005_b32.jsonl -- $BASE --batch-size 32 --synthetic-train-size 4800 --lr 0.05 --epochs 2 > $O/lr005_b32.log 2>&1
timeout -k 10 300 python -u scripts/trajectory_diff.py --out $O/lr01_b32.jsonl -- $BASE --batch-size 32 --synthetic-train-size 4800 --lr 0.1 --epochs 2 > $O/lr01_b32.log 2>&1
timeout -k 10 300 python -u scripts/trajectory_diff.py --out $O/lr01_b128.jsonl -- $BASE --batch-size 128 --synthetic-train-size 19200 --lr 0.1 --epochs 2 > $O/lr01_b128.log 2>&1
