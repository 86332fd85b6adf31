#!/bin/bash
# staged-epilogue read batching A/B (QB 8 for 256-row tiles = default build, vs the QB 4 build), isolated + in-step;
# then the two-stream graph capture repro (stops at the first failure)
set -o pipefail
O=${1:-gpurun_out/qb}
mkdir -p $O
ALT=imagent_amd/_native/ab/qb4/libimagent_kernels.so
for sh in 256,14,256,3,1 1024,14,256,1,1 512,7,512,3,1 256,28,512,1,1 2048,7,512,1,1; do
  timeout -k 10 180 python -u scripts/conv_bench.py --batch 2048 --bnb --only $sh >> $O/qb8.log 2>&1 || exit 1
  IMAGENT_KERNELS_LIB=$ALT timeout -k 10 180 python -u scripts/conv_bench.py --batch 2048 --bnb --only $sh >> $O/qb4.log 2>&1 || exit 1
done
for v in 8 4 8 4; do
  if [ $v = 4 ]; then L=$ALT; else L=; fi
  IMAGENT_KERNELS_LIB=$L timeout -k 10 300 python -u bench.py > $O/bench_$v.log 2>&1 || exit 1
  echo "qb=$v $(grep '"metric"' $O/bench_$v.log | cut -c60-130)" >> $O/bench_summary.log
done
timeout -k 10 240 python -u -X faulthandler scripts/graph_capture_repro.py --arch resnet18 --deterministic 1 --batch 64 > $O/graph_r18_det.log 2>&1; rc=$?; echo "rc=$rc" >> $O/graph_r18_det.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 240 python -u -X faulthandler scripts/graph_capture_repro.py --arch resnet50 --deterministic 0 --batch 128 > $O/graph_r50.log 2>&1; rc=$?; echo "rc=$rc" >> $O/graph_r50.log; [ $rc -eq 0 ] || exit 1
