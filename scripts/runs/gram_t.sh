#!/bin/bash
# isolated T = g^T h2 / G = h2^T h2 timings at the 4096-image default (scripts/gram_bench.py), every v3 stage shape
# and split count, torch.mm (hipBLASLt) as reference
set -o pipefail
O=${1:-gpurun_out/gramt}
mkdir -p $O
timeout -k 10 500 python -u scripts/gram_bench.py --batch 4096 --variants 0,-1,1,2,3,4,6 --splits 0,16,64,256 > $O/gram_4096.log 2>&1
