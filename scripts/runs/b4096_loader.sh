#!/bin/bash
# 4096-img/GPU readiness (large-tensor tests incl. the duplicated-batch training step), the GPU resize tests,
# the BN backward-apply grid / NT-load A/B (micro + in-step), bench at 2048 vs 4096 alternating, and the loader
# at 448^2 from 448^2 / 320^2 / 288^2 records on 8 concurrent ranks.
set -o pipefail
O=${1:-gpurun_out/b4096}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_resize_gpu.py tests/test_large_tensors_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for cfg in "8 0" "2 1" "4 1" "2 0"; do
  set -- $cfg
  IMAGENT_BN_APPLY_BPC=$1 IMAGENT_BN_NTLOAD=$2 timeout -k 10 300 python -u scripts/bn_bench.py --batch 2048 > $O/bnb_$1_$2.log 2>&1 || exit 1
done
for cfg in "8 0" "2 1" "8 0" "2 1" "4 1"; do
  set -- $cfg
  IMAGENT_BN_APPLY_BPC=$1 IMAGENT_BN_NTLOAD=$2 timeout -k 10 300 python -u bench.py > $O/bench_bn_$1_$2.log 2>&1 || exit 1
  echo "bpc=$1 ntl=$2 $(grep '"metric"' $O/bench_bn_$1_$2.log | cut -c1-120)" >> $O/bench_summary.log
done
for b in 2048 4096 2048 4096; do
  timeout -k 10 300 python -u bench.py --batch-size $b > $O/bench_$b.log 2>&1 || exit 1
  echo "b=$b $(grep '"metric"' $O/bench_$b.log | cut -c1-120) peak $(grep -o '"peak_hbm_gib": [0-9.]*' $O/bench_$b.log)" >> $O/bench_summary.log
done
timeout -k 10 600 python -u scripts/loader_bench.py --sizes 448,448@320,448@288 --ranks 8 --threads 2 --dir /tmp/imrec --out $O/loader.md > $O/loader.log 2>&1 || exit 1
