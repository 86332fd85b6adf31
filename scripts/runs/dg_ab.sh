#!/bin/bash
# BN backward apply: dgamma / dbeta accumulation spread over blocks (default) vs block 0 alone (ab/dg0 build):
# BN / block / kernel tests on the new build, then bench.py A/B at 256 and 4096 img
set -o pipefail
O=${1:-gpurun_out/dgab}
mkdir -p $O
OLD=$PWD/imagent-distributed-training-pytorch-with-slurm_amd/_native/ab/dg0/libimagent_kernels.so
timeout -k 10 600 python -u -m pytest tests/test_bn_numerics_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log >> $O/summary.log
run() { local tag=$1 lib=$2; shift 2; IMAGENT_KERNELS_LIB=$lib timeout -k 10 300 python -u bench.py "$@" > $O/$tag.log 2>&1 || exit 1; echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
run b256_new "" --batch-size 256 --steps 40 --warmup 10
run b256_old $OLD --batch-size 256 --steps 40 --warmup 10
run b256_new2 "" --batch-size 256 --steps 40 --warmup 10
run b256_old2 $OLD --batch-size 256 --steps 40 --warmup 10
run b4096_new "" --steps 12 --warmup 4
run b4096_old $OLD --steps 12 --warmup 4
timeout -k 10 300 python -u scripts/bn_bench.py --batch 256 > $O/bn256_new.log 2>&1 || exit 1
IMAGENT_KERNELS_LIB=$OLD timeout -k 10 300 python -u scripts/bn_bench.py --batch 256 > $O/bn256_old.log 2>&1 || exit 1
