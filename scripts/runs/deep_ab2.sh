#!/bin/bash
# 32-deep v3 rings for forward convs (IMAGENT_V3_DEEP=1) re-checked at the end-of-round HEAD, 4096 img
set -o pipefail
O=${1:-gpurun_out/deep2}
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 12 --warmup 4 > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
for i in 1 2 3; do
  run deep_$i IMAGENT_V3_DEEP=1
  run base_$i IMAGENT_X=0
done
