#!/bin/bash
# (1) BN passes at 256 img under rocprofv3 kernel-trace: kernel time vs the event timing of scripts/bn_bench.py
#     (whose small calls may be bounded by the Python launch path, not the GPU);
# (2) the two-stream graph at 256 img against ROCclr graph-execution knobs
set -o pipefail
O=${1:-gpurun_out/sbp}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bnprof -o run -- python3 scripts/bn_bench.py --batch 256 > $O/bn_bench_prof.log 2>&1 || exit 1
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --batch-size 256 --steps 40 --warmup 10 --graph 2 > $O/$tag.log 2>&1 || exit 1; echo "$tag $* $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
run g2_default IMAGENT_X=0
run g2_nopkt DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run g2_q1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1
run g2_q8 DEBUG_HIP_FORCE_GRAPH_QUEUES=8
run g2_default_b IMAGENT_X=0
