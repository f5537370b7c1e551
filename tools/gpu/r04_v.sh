#!/bin/bash
# round 4, call v: the device tracegen parity tests after the precompile_chip refactor, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_tracegen.py -m gpu -q --timeout 300 --timeout-method thread > $O/r04v_tracegen.log 2>&1 || { tail -60 $O/r04v_tracegen.log; exit 1; }
tail -2 $O/r04v_tracegen.log
timeout -k 10 900 python3 -u bench.py > $O/r04v_bench.json 2> $O/r04v_bench.err || { tail -40 $O/r04v_bench.err; exit 1; }
tail -c 300 $O/r04v_bench.json
