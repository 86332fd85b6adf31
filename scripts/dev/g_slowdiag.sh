# Diagnose the slow episodes: GPU clocks / temperature / power / memory / processes between bench runs
cd $GRAFT_REPO_ROOT
L=gpurun_out/slowdiag.log
: > $L
smi() { echo "--- smi $1 $(date +%T)" >> $L; timeout 30 rocm-smi --showtemp --showpower --showuse --showmemuse --showpids --showclocks 2>&1 | grep -v '^$' | grep -v '====' >> $L; timeout 30 amd-smi metric -p -c -t 2>/dev/null | head -n 60 >> $L; true; }
smi 0
for i in 1 2 3 4; do
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 2>/dev/null | grep '^{' | grep -o '"value": [0-9.]*\|"alloc_retries": [0-9]*' | tr '\n' ' ' >> $L || exit 1
  echo >> $L
  smi $i
done
