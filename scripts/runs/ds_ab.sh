#!/bin/bash
# downsample conv forward on the main stream (IMAGENT_DS_SIDE=0) vs beside the main chain on the side stream
set -o pipefail
O=${1:-gpurun_out/dsab}
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
B="--steps 12 --warmup 4"
run b4096_base IMAGENT_X=0
run b4096_ds0 IMAGENT_DS_SIDE=0
run b4096_base2 IMAGENT_X=0
run b4096_ds0b IMAGENT_DS_SIDE=0
B="--batch-size 256 --steps 40 --warmup 10"
run b256_base IMAGENT_X=0
run b256_ds0 IMAGENT_DS_SIDE=0
