#!/bin/bash
# the 16-wave weight-gradient grid: 256 blocks (one per CU) vs 192 / 128, in-step at 4096 img
set -o pipefail
O=${1:-gpurun_out/wtarget}
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 12 --warmup 4 > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
run t256 IMAGENT_X=0
run t192 IMAGENT_WGRAD_WIDE_TARGET=192
run t128 IMAGENT_WGRAD_WIDE_TARGET=128
run t256b IMAGENT_X=0
run t192b IMAGENT_WGRAD_WIDE_TARGET=192
run t128b IMAGENT_WGRAD_WIDE_TARGET=128
