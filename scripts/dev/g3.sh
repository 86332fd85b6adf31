set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/bn_bench.py --batch 512 > gpurun_out/bn512.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o c1 -- python3 scripts/conv_bench.py --batch 512 --only 64,56,256,1,1 > gpurun_out/prof_c1.log 2>&1
echo EXIT $?
