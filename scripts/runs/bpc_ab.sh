#!/bin/bash
# BN backward apply grid (blocks per CU) with the batched loads, in-step at 4096 img
set -o pipefail
O=${1:-gpurun_out/bpc}
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 12 --warmup 4 > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
run bpc4 IMAGENT_X=0
run bpc2 IMAGENT_BN_APPLY_BPC=2
run bpc8 IMAGENT_BN_APPLY_BPC=8
run bpc4b IMAGENT_X=0
run bpc2b IMAGENT_BN_APPLY_BPC=2
run bpc8b IMAGENT_BN_APPLY_BPC=8
