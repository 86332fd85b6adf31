set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc/a -o a -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmc/a.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc/b -o b -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmc/b.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace -d gpurun_out/pmc/c -o c -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmc/c.log 2>&1
echo EXIT $?
