#!/bin/bash
# The trainer GPU tests once, then the HBM streaming roof (profiles/hbm_roof.md).
set -o pipefail
O=${1:-gpurun_out/tr}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_trainer_gpu.py -x -v --timeout 600 --timeout-method thread > $O/trainer_tests.log 2>&1 || exit 1
hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/hbm_roof.hip -o /tmp/hbm_roof > $O/hbm_build.log 2>&1 || exit 1
timeout -k 10 300 /tmp/hbm_roof 4 > $O/hbm_roof.md 2>&1 || exit 1
