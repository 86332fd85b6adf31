#!/bin/bash
# the two-stream capture crash with native frames: single-stream graph tests first, then the two-stream one, in one
# process (the order that crashed); then the two-stream test alone in a fresh process. Stops at the first failure.
set -o pipefail
O=${1:-gpurun_out/gcrash}
mkdir -p $O
IMAGENT_SEGV_BT=1 timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k "graphed_two_stream_step_matches_eager and not deterministic" -v --timeout 200 --timeout-method thread > $O/alone.log 2>&1; rc=$?; echo "rc=$rc" >> $O/alone.log; [ $rc -eq 0 ] || exit 1
IMAGENT_SEGV_BT=1 timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k graphed -v --timeout 200 --timeout-method thread > $O/seq.log 2>&1; rc=$?; echo "rc=$rc" >> $O/seq.log; [ $rc -eq 0 ] || exit 1
