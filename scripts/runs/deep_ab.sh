#!/bin/bash
# v3 forward-ring A/B in-step (IMAGENT_V3_DEEP 1 vs 0, alternating) after the conv numerics tests
set -o pipefail
O=${1:-gpurun_out/deep}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv_shapes_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for v in 1 0 1 0; do
  IMAGENT_V3_DEEP=$v timeout -k 10 300 python -u bench.py > $O/bench_$v.log 2>&1 || exit 1
  echo "deep=$v $(grep '"metric"' $O/bench_$v.log | cut -c60-130)" >> $O/bench_summary.log
done
