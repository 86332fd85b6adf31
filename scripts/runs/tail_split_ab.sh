set -o pipefail
mkdir -p gpurun_out/tail
for v in 1 0 1 0 1 0; do
  IMAGENT_TAIL_SPLIT=$v timeout -k 10 240 python bench.py > gpurun_out/tail/bench_$v.log 2>&1 || exit 1
  echo "tail_split=$v $(grep '"metric"' gpurun_out/tail/bench_$v.log | cut -c60-120)" >> gpurun_out/tail/summary.log
done
