#!/bin/bash
# round 3 (session 2): bench with the maxshape-from-device-traces sub-leg, small then default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --log-n 18 --no-pmc --no-cpu-baseline --steps 2 > gpurun_out/r03r_small.json 2> gpurun_out/r03r_small.err || { tail -20 gpurun_out/r03r_small.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03r_small.json')); print(d['maxshape'].get('from_device_traces'))"
timeout -k 10 700 python3 -u bench.py > gpurun_out/r03r_bench.json 2> gpurun_out/r03r_bench.err || { tail -20 gpurun_out/r03r_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03r_bench.json'))
print(d['value'], d['ms_per_shard'], d['resident']['ms_per_shard'], d['serial_ms_per_shard'])
print(d['maxshape']['value'], d['maxshape']['resident'], d['maxshape'].get('from_device_traces'))"
