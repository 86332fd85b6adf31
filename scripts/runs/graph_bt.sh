#!/bin/bash
# the crashing two-stream capture (R18, 64 px, batch 8, no communicator: the test's configuration) in the repro, ONE
# GPU process: native backtrace on SIGSEGV (scripts/segv_bt.c) + HIP runtime log (AMD_LOG_LEVEL=3), last 600 KB kept
set -o pipefail
O=${1:-gpurun_out/gbt}
mkdir -p $O
AMD_LOG_LEVEL=3 timeout -k 10 240 python -u -X faulthandler scripts/graph_capture_repro.py --arch resnet18 --size 64 --batch 8 --comm local --deterministic 0 --steps 3 2>&1 | tail -c 600000 > $O/repro_tail.txt
echo "rc=$?" >> $O/repro_tail.txt
