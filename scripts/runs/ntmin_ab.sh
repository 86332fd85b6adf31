#!/bin/bash
# BN backward apply: plain loads below IMAGENT_BN_NTLOAD_MIN_MB (default 256) vs NT loads at every size (=0)
set -o pipefail
O=${1:-gpurun_out/ntmin}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bn_numerics_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log >> $O/summary.log
bb() { local tag=$1 mb=$2 b=$3; IMAGENT_BN_NTLOAD_MIN_MB=$mb timeout -k 10 300 python -u scripts/bn_bench.py --batch $b > $O/$tag.log 2>&1 || exit 1; echo "$tag $(grep 'per step' $O/$tag.log)" >> $O/summary.log; }
bb bn256_min256 256 256
bb bn256_min0 0 256
run() { local tag=$1 mb=$2; shift 2; IMAGENT_BN_NTLOAD_MIN_MB=$mb timeout -k 10 300 python -u bench.py "$@" > $O/$tag.log 2>&1 || exit 1; echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
run b256_min256 256 --batch-size 256 --steps 40 --warmup 10
run b256_min0 0 --batch-size 256 --steps 40 --warmup 10
run b256_min256b 256 --batch-size 256 --steps 40 --warmup 10
run b256_min0b 0 --batch-size 256 --steps 40 --warmup 10
run b4096_min256 256 --steps 12 --warmup 4
