set -o pipefail
mkdir -p gpurun_out
for v in 64 128 0; do
IMAGENT_STREAM_BNB=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b8_$v.log 2>&1 || exit 1
done
echo EXIT $?
