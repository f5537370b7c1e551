#!/bin/bash
# round 3 (session 2): the default bench line, then a rocprofv3 kernel trace of the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03l_bench.json 2> gpurun_out/r03l_bench.err || { tail -20 gpurun_out/r03l_bench.err; exit 1; }
tail -c 1500 gpurun_out/r03l_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03l_prof -o r03l -- python3 bench.py --steps 3 --warmup 1 --no-pmc --no-maxshape --no-cpu-baseline > gpurun_out/r03l_prof_bench.json 2> gpurun_out/r03l_prof.err || { tail -20 gpurun_out/r03l_prof.err; exit 1; }
find gpurun_out/r03l_prof -name "*stats*" | head
