#!/bin/bash
# the late round-6 defaults on the other bench configs (R152 1024 img, R18 448 512 img), same box: HEAD vs the
# downsample back on the side stream (IMAGENT_DS_SIDE=1) vs 1x1-only v3 weight gradients (IMAGENT_WGRAD_V3=1)
set -o pipefail
O=${1:-gpurun_out/other}
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
B="--arch resnet152 --batch-size 1024 --steps 12 --warmup 4"
run r152_head IMAGENT_X=0
run r152_ds1 IMAGENT_DS_SIDE=1
run r152_v1 IMAGENT_WGRAD_V3=1
run r152_head2 IMAGENT_X=0
B="--arch resnet18 --image-size 448 --batch-size 512 --steps 12 --warmup 4"
run r18_head IMAGENT_X=0
run r18_ds1 IMAGENT_DS_SIDE=1
run r18_v1 IMAGENT_WGRAD_V3=1
run r18_head2 IMAGENT_X=0
