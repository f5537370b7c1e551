set -e
mkdir -p gpurun_out
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t5.log 2>&1 || { tail -40 gpurun_out/t5.log; exit 1; }
tail -2 gpurun_out/t5.log
timeout -k 10 600 python bench.py > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { tail -30 gpurun_out/bench5.err; exit 1; }
cat gpurun_out/bench5.json
