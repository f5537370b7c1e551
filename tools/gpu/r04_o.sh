#!/bin/bash
# round 4, call o: the whole GPU test suite with this round's changes, then smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/r04o_gpu_tests.log 2>&1 || { tail -40 $O/r04o_gpu_tests.log; exit 1; }
tail -3 $O/r04o_gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/r04o_smoke.log 2>&1 || { tail -20 $O/r04o_smoke.log; exit 1; }
tail -3 $O/r04o_smoke.log
