# bench.py at 2^20..2^23 rows (BASELINE: 2^20-2^24; 2^24 exceeds the two-adicity at blowup 2)
set -e
mkdir -p gpurun_out
: > gpurun_out/size_sweep.jsonl
for lg in 20 21 22 23; do
  timeout -k 10 300 python bench.py --log-n $lg --no-cpu-baseline --steps 3 >> gpurun_out/size_sweep.jsonl 2> gpurun_out/size_sweep_$lg.err || { tail -20 gpurun_out/size_sweep_$lg.err; exit 1; }
  tail -1 gpurun_out/size_sweep.jsonl | cut -c1-200
done
