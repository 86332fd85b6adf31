#!/bin/bash
# stem pool passes in isolation (scripts/pool_bench.py) at 4096 img: plain vs non-temporal backward stores
set -o pipefail
O=${1:-gpurun_out/poolab}
mkdir -p $O
for nt in 0 1 0 1; do
  IMAGENT_POOL_NT=$nt timeout -k 10 300 python -u scripts/pool_bench.py --batch 4096 >> $O/pool.log 2>&1 || exit 1
done
