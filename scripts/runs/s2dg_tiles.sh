set -o pipefail
mkdir -p gpurun_out/s2dg
for sh in 128,56,128,3,2 256,28,256,3,2 512,14,512,3,2; do
  timeout -k 10 120 python -u scripts/conv_bench.py --batch 2048 --bnb --only $sh --tiles 2,4,8,17,18 >> gpurun_out/s2dg/conv.log 2>&1 || exit 1
done
