#!/bin/bash
# round 3 (session 2): tracegen GPU tests (ShaExtend added)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_tracegen.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03o_tracegen.log 2>&1 || { tail -40 gpurun_out/r03o_tracegen.log; exit 1; }
tail -2 gpurun_out/r03o_tracegen.log
