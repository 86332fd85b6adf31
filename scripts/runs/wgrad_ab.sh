#!/bin/bash
# 1x1 weight-gradient stage shapes in-step (IMAGENT_WGRAD_V3 1: 64 rows x 2 stages, 2: 64 x 3, 3: 32 x 4), alternating
set -o pipefail
O=${1:-gpurun_out/wgab}
mkdir -p $O
for v in 1 2 3 1 2 3; do
  IMAGENT_WGRAD_V3=$v timeout -k 10 300 python -u bench.py > $O/bench_$v.log 2>&1 || exit 1
  echo "wgrad_v3=$v $(grep '"metric"' $O/bench_$v.log | cut -c60-130)" >> $O/bench_summary.log
done
timeout -k 10 300 python -u scripts/bn_bench.py --batch 256 > $O/bn_bench_256.log 2>&1 || exit 1
