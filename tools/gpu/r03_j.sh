#!/bin/bash
# round 3 (session 2): KeccakSponge on the GPU, then the whole -m gpu suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_keccak.py -m gpu -x -v --timeout 380 --timeout-method thread > gpurun_out/r03j_keccak.log 2>&1 || { tail -30 gpurun_out/r03j_keccak.log; exit 1; }
tail -3 gpurun_out/r03j_keccak.log
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --deselect tests/test_keccak.py::test_gpu_keccak_execution_bytes_identical > gpurun_out/r03j_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r03j_tests.log
exit $rc
