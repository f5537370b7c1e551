#!/bin/bash
# round 3 (session 2): the -m gpu suite (device tracegen for Bitwise/Lt/shifts/Branch/MemoryInstrs),
# the default bench line, a kernel-trace profile of the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_tracegen.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03k_tracegen.log 2>&1 || { tail -30 gpurun_out/r03k_tracegen.log; exit 1; }
tail -2 gpurun_out/r03k_tracegen.log
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --deselect tests/test_keccak.py::test_gpu_keccak_execution_bytes_identical --ignore tests/test_tracegen.py > gpurun_out/r03k_tests.log 2>&1 || { tail -30 gpurun_out/r03k_tests.log; exit 1; }
tail -2 gpurun_out/r03k_tests.log
