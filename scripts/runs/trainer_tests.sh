#!/bin/bash
set -o pipefail
O=${1:-gpurun_out/trainer}
mkdir -p $O
timeout -k 10 850 python -u -m pytest tests/test_trainer_gpu.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
