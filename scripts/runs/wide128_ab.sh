set -o pipefail
mkdir -p gpurun_out/w128
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "test_conv_v3" -x -q --timeout 120 --timeout-method thread > gpurun_out/w128/test.log 2>&1 || exit 1
for sh in 128,28,128,3,1 128,56,128,3,2 128,28,512,1,1 512,28,128,1,1; do
  timeout -k 10 120 python -u scripts/conv_bench.py --batch 2048 --bnb --only $sh --tiles 18,19 >> gpurun_out/w128/conv.log 2>&1 || exit 1
done
for v in 0 1 0 1; do
  IMAGENT_V3_WIDE128=$v timeout -k 10 240 python bench.py > gpurun_out/w128/bench_$v.log 2>&1 || exit 1
  echo "wide128=$v $(tail -1 gpurun_out/w128/bench_$v.log | cut -c1-140)" >> gpurun_out/w128/bench_summary.log
done
