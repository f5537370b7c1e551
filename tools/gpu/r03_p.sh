#!/bin/bash
# round 3 (session 2) final evidence: the whole -m gpu suite, the default bench line, a rocprofv3 kernel
# trace of the headline (csv), the tracegen bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03p_tests.log 2>&1 || { tail -30 gpurun_out/r03p_tests.log; exit 1; }
tail -2 gpurun_out/r03p_tests.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03p_bench.json 2> gpurun_out/r03p_bench.err || { tail -20 gpurun_out/r03p_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03p_bench.json'))
print(d['value'], d['ms_per_shard'], d['resident'], d['serial_ms_per_shard'], d['roofline']['frac'], d['maxshape']['value'], d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03p_prof -o r03p -- python3 bench.py --steps 3 --warmup 1 --no-pmc --no-maxshape --no-cpu-baseline --inflight 1 > gpurun_out/r03p_prof_bench.json 2> gpurun_out/r03p_prof.err || { tail -20 gpurun_out/r03p_prof.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --workload tracegen --steps 5 --warmup 1 > gpurun_out/r03p_tracegen_bench.json 2> gpurun_out/r03p_tracegen_bench.err || { tail -20 gpurun_out/r03p_tracegen_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03p_tracegen_bench.json'))
for k, v in d['chips'].items(): print(k, v['rows'], v['ms'], v['GBps'], v['frac_of_hbm_peak'])"
