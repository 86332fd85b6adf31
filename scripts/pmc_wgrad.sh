#!/bin/bash
# PMC passes over scripts/wgrad_ab.py on ONE weight-gradient shape and variant list (main-loop diagnosis):
#   gpurun -- bash scripts/pmc_wgrad.sh TAG "Ci,H,Co,k,s" "variants" [batch]
# Each rocprofv3 pass has its own time limit; the script stops at the first failure.
set -e
tag=$1; shape=$2; vars=${3:--1,1}; batch=${4:-1024}
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
D=$R/gpurun_out/pmcw_$tag
mkdir -p $D
run() {
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d $D/$1 -o p --output-format rocpd \
        -- python3 $R/scripts/wgrad_ab.py --batch $batch --only $shape --variants=$vars --reps 3 > $D/$1.log 2>&1
}
run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE
cd $R
for p in $D/*/; do python3 scripts/pmc_kernels.py $(ls $p/*.db | head -1) ; done > $D/summary.txt
