#!/bin/bash
# second round of the downsample-stream A/B at 4096 img (three more alternating pairs)
set -o pipefail
O=${1:-gpurun_out/dsab2}
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 12 --warmup 4 > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
for i in 1 2 3; do
  run ds0_$i IMAGENT_DS_SIDE=0
  run base_$i IMAGENT_X=0
done
