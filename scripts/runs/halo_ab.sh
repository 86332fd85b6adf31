#!/bin/bash
# with the v3 weight-gradient default (6): the wide 3x3 halo wgrads (128 @28, 256 @14) on the LDS-DMA v3 loop
# instead (IMAGENT_WGRAD_HALO=1: halo kernel for 64 -> 64 only), in-step A/B
set -o pipefail
O=${1:-gpurun_out/haloab}
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
B="--steps 12 --warmup 4"
run b4096_base IMAGENT_X=0
run b4096_h1 IMAGENT_WGRAD_HALO=1
run b4096_base2 IMAGENT_X=0
run b4096_h1b IMAGENT_WGRAD_HALO=1
B="--batch-size 256 --steps 40 --warmup 10"
run b256_base IMAGENT_X=0
run b256_h1 IMAGENT_WGRAD_HALO=1
