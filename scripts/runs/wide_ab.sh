#!/bin/bash
# the 256 x 256 weight-gradient tile for shapes of >= IMAGENT_WGRAD_WIDE_MIN_ROWS output pixels: default (200,704)
# vs off, at 4096 img, and the threshold at 256 img (stages 1-2 / stage 1 / none wide)
set -o pipefail
O=${1:-gpurun_out/wide}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k wgrad -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log >> $O/summary.log
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
B="--steps 12 --warmup 4"
run b4096_def IMAGENT_X=0
run b4096_off IMAGENT_WGRAD_WIDE_MIN_ROWS=999999999
run b4096_def2 IMAGENT_X=0
B="--batch-size 256 --steps 40 --warmup 10"
run b256_def IMAGENT_X=0
run b256_off IMAGENT_WGRAD_WIDE_MIN_ROWS=999999999
run b256_800k IMAGENT_WGRAD_WIDE_MIN_ROWS=802816
run b256_def2 IMAGENT_X=0
run b256_off2 IMAGENT_WGRAD_WIDE_MIN_ROWS=999999999
