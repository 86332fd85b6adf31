#!/bin/bash
# Three rocprofv3 --pmc passes over a short bench run (one pass per counter group:
# rocprofv3 does not split counters over passes), then the per-kernel table.
#   gpurun -- bash scripts/pmc_passes.sh OUT.md [bench args...]
# Each pass is bounded by its own time limit; the script stops at the first failure.
set -e
out=${1:-profiles/pmc.md}
shift || true
args=${@:---steps 3 --warmup 2}
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
P=${PMC_DIR:-$R/gpurun_out/pmc}
mkdir -p $P
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $P/p1 -o p1 --output-format rocpd \
    -- python3 $R/bench.py $args
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES -d $P/p2 -o p2 --output-format rocpd \
    -- python3 $R/bench.py $args
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d $P/p3 -o p3 \
    --output-format rocpd -- python3 $R/bench.py $args
cd $R
python3 scripts/pmc_summary.py $out $(ls $P/p1/*.db | head -1) $(ls $P/p2/*.db | head -1) \
    $(ls $P/p3/*.db | head -1)
