#!/bin/bash
# round 4, call b: the whole -m gpu suite (LogUp kernel with LDS-staged numerators/prefix products, the
# compress tree over MIPS leaves, the tendermint execution on the reference's blocks)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r04b_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04b_gpu_tests.log; exit 1; }
tail -4 gpurun_out/r04b_gpu_tests.log
