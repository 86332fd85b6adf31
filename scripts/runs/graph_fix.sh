#!/bin/bash
# two-stream capture after the self-wait fix (streams.wait: a stream never waits on itself): the test that crashed
# (alone), every graph test, then R50 at 256 img eager vs --graph 1 vs --graph 2 (alternating)
set -o pipefail
O=${1:-gpurun_out/gfix2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k "graphed_two_stream_step_matches_eager and not deterministic" -v --timeout 200 --timeout-method thread > $O/alone.log 2>&1; rc=$?; echo "rc=$rc" >> $O/alone.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k graphed -v --timeout 200 --timeout-method thread > $O/seq.log 2>&1; rc=$?; echo "rc=$rc" >> $O/seq.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for g in 0 1 2; do
    timeout -k 10 300 python -u bench.py --batch-size 256 --steps 40 --warmup 5 --graph $g > $O/b256_g${g}_$r.log 2>&1 || exit 1
    echo "graph=$g $(grep '"metric"' $O/b256_g${g}_$r.log | cut -c60-130)" >> $O/bench_summary.log
  done
done
