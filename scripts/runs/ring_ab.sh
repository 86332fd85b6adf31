#!/bin/bash
# v3 ring-depth A/B (round 6): explicit tiles on the long-K R50 shapes, isolated (scripts/conv_bench.py --tiles)
set -o pipefail
O=${1:-gpurun_out/ring}
mkdir -p $O
for sh in 256,14,256,3,1 1024,14,256,1,1 512,7,512,3,1 512,14,512,3,2 256,28,256,3,2; do
  timeout -k 10 180 python -u scripts/conv_bench.py --batch 2048 --bnb --only $sh --tiles 17,29,30 >> $O/big.log 2>&1 || exit 1
done
for sh in 128,28,128,3,1 512,28,128,1,1 128,56,128,3,2; do
  timeout -k 10 180 python -u scripts/conv_bench.py --batch 2048 --bnb --only $sh --tiles 18,31,32 >> $O/small.log 2>&1 || exit 1
done
