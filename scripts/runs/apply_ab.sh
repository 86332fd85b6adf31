#!/bin/bash
# BN backward apply with its U rows' loads pinned ahead of the math (default) vs the compiler's one-row-in-flight
# schedule (ab/serial: -DIMAGENT_BN_APPLY_SERIAL): tests, isolated passes at 256 / 2048 img, bench.py at 256 / 4096
set -o pipefail
O=${1:-gpurun_out/applyab}
mkdir -p $O
OLD=$PWD/imagent-distributed-training-pytorch-with-slurm_amd/_native/ab/serial/libimagent_kernels.so
timeout -k 10 600 python -u -m pytest tests/test_bn_numerics_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log >> $O/summary.log
bb() { local tag=$1 lib=$2 b=$3; IMAGENT_KERNELS_LIB=$lib timeout -k 10 300 python -u scripts/bn_bench.py --batch $b > $O/$tag.log 2>&1 || exit 1; echo "$tag $(grep 'per step' $O/$tag.log)" >> $O/summary.log; }
bb bn256_new "" 256
bb bn256_old $OLD 256
bb bn2048_new "" 2048
bb bn2048_old $OLD 2048
run() { local tag=$1 lib=$2; shift 2; IMAGENT_KERNELS_LIB=$lib timeout -k 10 300 python -u bench.py "$@" > $O/$tag.log 2>&1 || exit 1; echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
run b256_new "" --batch-size 256 --steps 40 --warmup 10
run b256_old $OLD --batch-size 256 --steps 40 --warmup 10
run b4096_new "" --steps 12 --warmup 4
run b4096_old $OLD --steps 12 --warmup 4
run b256_new2 "" --batch-size 256 --steps 40 --warmup 10
run b4096_new2 "" --steps 12 --warmup 4
run b4096_old2 $OLD --steps 12 --warmup 4
