#!/bin/bash
# IMAGENT_WGRAD_V3=7: the 16-wave 256 x 256 weight-gradient tile wherever it covers the shape (incl. the Gram T)
set -o pipefail
O=${1:-gpurun_out/wgv7}
mkdir -p $O
IMAGENT_WGRAD_V3=7 timeout -k 10 900 python -u -m pytest tests/test_conv_shapes_gpu.py -k production -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log >> $O/summary.log
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
B="--steps 12 --warmup 4"
run b4096_base IMAGENT_X=0
run b4096_v7 IMAGENT_WGRAD_V3=7
run b4096_base2 IMAGENT_X=0
run b4096_v7b IMAGENT_WGRAD_V3=7
B="--batch-size 256 --steps 40 --warmup 10"
run b256_base IMAGENT_X=0
run b256_v7 IMAGENT_WGRAD_V3=7
