set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3 4; do timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py tests/test_model_gpu.py -q -s -k "two_ranks or graphed" --timeout 120 --timeout-method thread > gpurun_out/t16_$i.log 2>&1; echo "run $i rc=$? $(grep -o "graph-vs-eager.*" gpurun_out/t16_$i.log) $(tail -1 gpurun_out/t16_$i.log)"; done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b16.log 2>&1
echo EXIT $?
