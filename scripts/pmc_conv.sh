#!/bin/bash
# PMC passes over conv_bench.py on ONE conv shape (kernel main-loop diagnosis):
#   gpurun -- bash scripts/pmc_conv.sh TAG "Ci,H,Co,k,s" "tiles"
# Each rocprofv3 pass has its own time limit; the script stops at the first failure.
set -e
tag=$1; shape=$2; tiles=${3:-8}
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
D=$R/gpurun_out/pmc_$tag
mkdir -p $D
[ -f $R/gpurun_out/rocprof_counters.txt ] || timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/rocprof_counters.txt 2>&1 || true
run() {
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d $D/$1 -o p --output-format rocpd \
        -- python3 $R/scripts/conv_bench.py --batch 1024 --only $shape --tiles $tiles > $D/$1.log 2>&1
}
run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE
cd $R
for p in $D/*/; do python3 scripts/pmc_kernels.py $(ls $p/*.db | head -1) ; done > $D/summary.txt
