#!/bin/bash
# Per-stream kernel tables of the headline step: rocprofv3 --kernel-trace over bench.py, then
# scripts/stream_timeline.py. Usage (GPU box): bash scripts/runs/stream_tables.sh [TAG] [bench args...]
# (round-5 drivers _r5i / _r5q / _r8v / _prof_final were this script with different bench args / --kernels N)
set -o pipefail
TAG=${1:-stream}; shift || true
ARGS=${@:---steps 4 --warmup 2}
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 $R/bench.py $ARGS > $O/bench.log 2>&1 || exit 1
cd $R
DB=$(find $O/db -name "*results.db" | head -1)
python scripts/stream_timeline.py $DB --kernels 80 > $O/stream_tables.md 2>&1 || exit 1
find $O/db -name "*.db" -delete
