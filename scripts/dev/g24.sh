mkdir -p gpurun_out
for i in 1 2 3 4; do
  (rocm-smi --showtemp --showpower --showclocks 2>/dev/null | grep -E "Temperature|Power|sclk|mclk|fclk" | head -8) > gpurun_out/smi_$i.txt
  timeout -k 10 300 python -u bench.py > gpurun_out/b24_$i.log 2>&1 || exit 1
  echo "run $i $(tail -1 gpurun_out/b24_$i.log | cut -c60-110)"
done
(rocm-smi --showtemp --showpower --showclocks 2>/dev/null | grep -E "Temperature|Power|sclk|mclk|fclk" | head -8) > gpurun_out/smi_5.txt
echo done
