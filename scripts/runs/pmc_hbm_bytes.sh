#!/bin/bash
# HBM bytes per kernel of the headline step (profiles/r50_b2048_r5_hbm_bytes.md): two rocprofv3 PMC passes
# (FETCH_SIZE, then WRITE_SIZE; one counter group per pass), tabulated by scripts/pmc_bytes_table.py.
# Usage (GPU box): bash scripts/runs/pmc_hbm_bytes.sh [TAG] [bench args...]   (round-5 drivers _r8p / _r8q)
set -o pipefail
TAG=${1:-pmc_bytes}; shift || true
ARGS=${@:---steps 2 --warmup 1}
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/f -o f --output-format rocpd -- python3 $R/bench.py $ARGS > $O/f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/w -o w --output-format rocpd -- python3 $R/bench.py $ARGS > $O/w.log 2>&1 || exit 1
cd $R
python3 scripts/pmc_bytes_table.py $(ls $O/f/*.db | head -1) $(ls $O/w/*.db | head -1) > $O/hbm_bytes.md || exit 1
