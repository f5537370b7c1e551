set -e
mkdir -p gpurun_out
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t7.log 2>&1 || { tail -40 gpurun_out/t7.log; exit 1; }
tail -2 gpurun_out/t7.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench7.json 2> gpurun_out/bench7.err || { tail -30 gpurun_out/bench7.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench7.json')); print(d['value'], d['ms_per_step']); print(json.dumps(d['stages_ms_per_step']))"
