set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pfinal
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pfinal/db -o run -- python3 $R/bench.py --steps 4 --warmup 2 > $R/gpurun_out/pfinal/bench.log 2>&1 || exit 1
cd $R
DB=$(find gpurun_out/pfinal/db -name "*results.db" | head -1)
python scripts/stream_timeline.py $DB --kernels 60 > gpurun_out/pfinal/stream_tables.md 2>&1 || exit 1
find gpurun_out/pfinal/db -name "*.db" -delete
