mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b25_$i.log 2>&1
  echo "run $i rc=$? $(tail -1 gpurun_out/b25_$i.log | cut -c60-100)"
  sleep 2
  echo "-- pids using the GPU after run $i:"; rocm-smi --showpids 2>/dev/null | grep -v "^=" | head -8
  echo "-- my processes:"; ps -u $(id -u) -o pid,ppid,stat,etime,cmd | grep -v "ps -u" | head -12
done
