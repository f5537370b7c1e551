#!/bin/bash
# round 5, call r: the driver's commands on HEAD -- the whole -m gpu suite, smoke(), then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1200 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=15 > $O/r05r_gpu_tests.log 2>&1 || { tail -60 $O/r05r_gpu_tests.log; exit 1; }
tail -3 $O/r05r_gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r05r_smoke.log 2>&1 || { tail -30 $O/r05r_smoke.log; exit 1; }
tail -1 $O/r05r_smoke.log
timeout -k 10 1200 python3 -u bench.py > $O/r05r_bench.json 2> $O/r05r_bench.err || { tail -40 $O/r05r_bench.err; exit 1; }
tail -c 600 $O/r05r_bench.json
