#!/bin/bash
# production-shape test with the band stem, then convergence on the 'mix' task (overlapping class Gaussians):
# hip bf16, Gram everywhere, fp8 Gram everywhere, fp32 PyTorch oracle
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r5h; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_conv_shapes_gpu.py -m gpu > $O/shapes.log 2>&1 || { echo shapes failed; tail -40 $O/shapes.log; exit 1; }
tail -3 $O/shapes.log
timeout -k 10 850 python -u scripts/convergence.py --arch resnet50 --classes 100 --epochs 8 --batch-size 128 --steps-per-epoch 400 --image-size 64 --task mix --paths gram,fp8 --timeout 300 --out $O/convergence_mix_r50.md > $O/conv.log 2>&1; rc=$?
echo "rc=$rc"; tail -30 $O/conv.log
