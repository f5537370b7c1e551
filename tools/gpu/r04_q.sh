#!/bin/bash
# round 4, call q: the default bench line with the register-weight openings and the compress node templates
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python3 -u bench.py > $O/r04q_bench.log 2>&1 || { tail -30 $O/r04q_bench.log; exit 1; }
tail -1 $O/r04q_bench.log | cut -c1-300
