set -o pipefail
mkdir -p gpurun_out
for w in 0 1 32 64; do IMAGENT_WGRAD_WIDE=$w timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 > gpurun_out/c21_$w.log 2>&1 || exit 1; done
IMAGENT_WGRAD_WIDE=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad or conv_fwd_dgrad" --timeout 120 --timeout-method thread > gpurun_out/t21.log 2>&1
echo EXIT $?
