#!/bin/bash
# BN backward apply at 256 img: what sets its ~20 us per-call floor (in-pass fold, NT loads, grid)
set -o pipefail
O=${1:-gpurun_out/bnsmall}
mkdir -p $O
b() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u scripts/bn_bench.py --batch 256 > $O/$tag.log 2>&1 || exit 1; }
b base IMAGENT_X=0
b nofold IMAGENT_BN_FOLD_IN=0
b ntl0 IMAGENT_BN_NTLOAD=0
b bpc8 IMAGENT_BN_APPLY_BPC=8
b bpc1 IMAGENT_BN_APPLY_BPC=1
