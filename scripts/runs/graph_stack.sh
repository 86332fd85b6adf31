#!/bin/bash
# is the EndCapture crash a DEEP (finite) recursion or an infinite one? The same single repro process with a 1 GiB
# main-thread stack (ulimit -s): deep -> it completes; infinite -> it still segfaults (bounded by the 1 GiB)
set -o pipefail
O=${1:-gpurun_out/gstack}
mkdir -p $O
ulimit -s 1048576
timeout -k 10 240 python -u -X faulthandler scripts/graph_capture_repro.py --arch resnet18 --size 64 --batch 8 --comm local --deterministic 0 --steps 6 > $O/repro_bigstack.log 2>&1; rc=$?; echo "rc=$rc" >> $O/repro_bigstack.log
