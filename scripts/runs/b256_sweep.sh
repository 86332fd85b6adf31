#!/bin/bash
# 256 img/GPU: in-step A/B of the switches whose defaults were tuned at 1024-4096 img
set -o pipefail
O=${1:-gpurun_out/b256sw}
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --batch-size 256 --steps 40 --warmup 10 > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
run base IMAGENT_X=0
run deep IMAGENT_V3_DEEP=1
run gram40k IMAGENT_GRAM_MIN_ROWS=40000
run gram300k IMAGENT_GRAM_MIN_ROWS=300000
run nogram IMAGENT_BN_GRAM=0
run noxfuse IMAGENT_BN_XFUSE=0
run bpc8 IMAGENT_BN_APPLY_BPC=8
run inflight4 IMAGENT_MAX_INFLIGHT=4
run base_b IMAGENT_X=0
