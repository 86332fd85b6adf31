#!/bin/bash
# the 4-pixel normalize kernel: its tests + the data / model tests that feed through it, then bench.py at HEAD
set -o pipefail
O=${1:-gpurun_out/norm}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_resize_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log >> $O/summary.log
run() { local tag=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$tag.log 2>&1 || exit 1; echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
run b4096_a --steps 20 --warmup 5
run b256 --batch-size 256 --steps 40 --warmup 10
run b4096_b --steps 20 --warmup 5
