#!/bin/bash
# the step on a high-priority stream (IMAGENT_MAIN_PRIO=1) vs the default stream, 4096 and 256 img
set -o pipefail
O=${1:-gpurun_out/prio}
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
B="--steps 12 --warmup 4"
run b4096_base IMAGENT_X=0
run b4096_prio IMAGENT_MAIN_PRIO=1
run b4096_base2 IMAGENT_X=0
run b4096_prio2 IMAGENT_MAIN_PRIO=1
B="--batch-size 256 --steps 40 --warmup 10"
run b256_base IMAGENT_X=0
run b256_prio IMAGENT_MAIN_PRIO=1
