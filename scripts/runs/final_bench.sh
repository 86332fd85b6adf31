#!/bin/bash
# end-of-round benches at HEAD: the driver's default command twice, 2048 img, ResNet-152 (config 4 per GPU),
# ResNet-18 at 448 (the reference's own run), eval throughput
set -o pipefail
O=${1:-gpurun_out/fbench6}
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$tag.log 2>&1 || exit 1; echo "$tag $(grep '"metric"' $O/$tag.log | cut -c1-160)" >> $O/summary.log; }
run default_1 --gpus 1 --steps 20 --warmup 5
run default_2 --gpus 1 --steps 20 --warmup 5
run b2048 --batch-size 2048
run r152_b1024 --arch resnet152 --batch-size 1024
run r18_448_b512 --arch resnet18 --image-size 448 --batch-size 512
run eval_b2048 --batch-size 2048 --eval 10
run fp8_b2048 --batch-size 2048 --dtype fp8
run b256_eager --batch-size 256 --steps 30 --warmup 10
run b256_graph2 --batch-size 256 --steps 30 --warmup 10 --graph 2
