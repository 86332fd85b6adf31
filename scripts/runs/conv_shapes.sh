#!/bin/bash
# Per-shape conv directions at the headline batch (profiles/r50_b2048_r5_conv_shapes.md):
# the auto-dispatched kernel per direction, then the hipBLASLt plain-GEMM comparison (--blas).
# Usage (GPU box): bash scripts/runs/conv_shapes.sh [TAG] [batch]   (round-5 drivers _r6d / _r5w)
set -o pipefail
TAG=${1:-conv_shapes}; B=${2:-2048}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u scripts/conv_bench.py --batch $B --bnb > $O/conv.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/conv_bench.py --batch $B --blas > $O/blas.log 2>&1 || exit 1
