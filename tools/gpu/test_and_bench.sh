set -e
mkdir -p gpurun_out
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t8.log 2>&1 || { tail -40 gpurun_out/t8.log; exit 1; }
tail -2 gpurun_out/t8.log
timeout -k 10 600 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/bench8.json 2> gpurun_out/bench8.err || { tail -30 gpurun_out/bench8.err; exit 1; }
cat gpurun_out/bench8.json
ZKM_NO_JIT=1 timeout -k 10 600 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/bench8b.json 2> gpurun_out/bench8b.err || { tail -30 gpurun_out/bench8b.err; exit 1; }
cat gpurun_out/bench8b.json
