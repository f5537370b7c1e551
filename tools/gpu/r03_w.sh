#!/bin/bash
# round 3 (session 2): final evidence after the LDE batching change: full GPU suite, default bench, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03w_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03w_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03w_gpu_tests.log
timeout -k 10 700 python3 -u bench.py > gpurun_out/r03w_bench.json 2> gpurun_out/r03w_bench.err || { tail -20 gpurun_out/r03w_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03w_bench.json'))
print(d['value'], d['ms_per_shard'], d['resident']['ms_per_shard'], d['serial_ms_per_shard'], d['roofline'])"
