#!/bin/bash
# two-stream HIP graph: the graph-vs-eager tests, then R50 at 256 img/GPU eager vs --graph 1 vs --graph 2 (alternating)
set -o pipefail
O=${1:-gpurun_out/graph}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -k graphed -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for g in 0 1 2; do
    timeout -k 10 300 python -u bench.py --batch-size 256 --steps 40 --warmup 5 --graph $g > $O/b256_g${g}_$r.log 2>&1 || exit 1
    echo "graph=$g $(grep '"metric"' $O/b256_g${g}_$r.log | cut -c60-130)" >> $O/bench_summary.log
  done
done
