#!/bin/bash
# PMC passes over scripts/gram_dgrad_bench.py (layer 1's conv3 dgrad family on the streaming kernel: plain, with the
# BN-backward epilogue, and the Gram form over [g | h2]) -- why the Gram form streams at ~3.2 TB/s in-step.
# One rocprofv3 run per counter pass, each under its own time limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
D=$R/${1:-gpurun_out/pmc_gd}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/scripts/gram_dgrad_bench.py --batch 1024 --reps 5 > $D/plain_timing.log 2>&1 || exit 1
run() {
    local tag=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d $D/$tag -o p --output-format rocpd \
        -- python3 $R/scripts/gram_dgrad_bench.py --batch 1024 --reps 5 > $D/$tag.log 2>&1 || exit 1
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run p2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run p3 FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE
cd $R
for p in $D/p*/; do python3 scripts/pmc_kernels.py $(ls $p/*.db | head -1); done > $D/summary.txt 2>&1
