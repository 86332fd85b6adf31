set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
 (cd _old && timeout -k 10 200 python -u -m pytest tests/test_multirank_gpu.py -q -s --timeout 120 --timeout-method thread 2>&1 | grep -E "ERR|passed|failed") 
 timeout -k 10 200 python -u -m pytest tests/test_multirank_gpu.py -q -s --timeout 120 --timeout-method thread 2>&1 | grep -E "ERR|passed|failed" | sed 's/^/NEW /'
done
echo done
