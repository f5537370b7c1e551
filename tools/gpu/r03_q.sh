#!/bin/bash
# round 3 (session 2): tracegen after the inversion / flag-table changes: GPU tests + tracegen bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_tracegen.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03q_tracegen.log 2>&1 || { tail -40 gpurun_out/r03q_tracegen.log; exit 1; }
tail -2 gpurun_out/r03q_tracegen.log
timeout -k 10 300 python3 -u bench.py --workload tracegen --steps 5 --warmup 1 > gpurun_out/r03q_tracegen_bench.json 2> gpurun_out/r03q_tracegen_bench.err || { tail -20 gpurun_out/r03q_tracegen_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03q_tracegen_bench.json'))
for k, v in d['chips'].items(): print(k, v['rows'], v['ms'], v['GBps'], v['frac_of_hbm_peak'])"
