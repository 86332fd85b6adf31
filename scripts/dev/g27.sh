set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t27.log 2>&1 && \
echo "tests: $(tail -1 gpurun_out/t27.log)" && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke27.log 2>&1 && \
echo "smoke: $(tail -1 gpurun_out/smoke27.log)" && \
timeout -k 10 300 python -u bench.py > gpurun_out/b27_1.log 2>&1 && \
echo "bench: $(tail -1 gpurun_out/b27_1.log | cut -c1-200)" && \
timeout -k 10 300 python -u bench.py --batch-size 1024 --steps 10 --warmup 3 > gpurun_out/b27_2.log 2>&1 && \
echo "bench1024: $(tail -1 gpurun_out/b27_2.log | cut -c1-200)"
