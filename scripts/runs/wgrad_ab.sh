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
# two-stream graph capture repro (R18 deterministic, the round-1 / round-5 crash config; then R50 non-deterministic)
timeout -k 10 240 python -u -X faulthandler scripts/graph_capture_repro.py --arch resnet18 --deterministic 1 --batch 64 > $O/graph_r18_det.log 2>&1; rc=$?; echo "rc=$rc" >> $O/graph_r18_det.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 240 python -u -X faulthandler scripts/graph_capture_repro.py --arch resnet50 --deterministic 0 --batch 128 > $O/graph_r50.log 2>&1; rc=$?; echo "rc=$rc" >> $O/graph_r50.log; [ $rc -eq 0 ] || exit 1
