#!/bin/bash
# round 5, call a: the driver's exact GPU-test command on HEAD (priority-ordered suite), then smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests/ -x -q -m gpu -v --timeout 600 --timeout-method thread > $O/r05a_gpu_tests.log 2>&1 || { tail -60 $O/r05a_gpu_tests.log; exit 1; }
tail -3 $O/r05a_gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/r05a_smoke.log 2>&1 || { tail -40 $O/r05a_smoke.log; exit 1; }
cat $O/r05a_smoke.log | tail -3
