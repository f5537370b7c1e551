#!/bin/bash
# round 4, call s: the Poseidon2Permute device trace (and the recursion Poseidon2 kernel on the shared row code)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_tracegen.py tests/test_recursion.py tests/test_compress_tree.py -m gpu -v --timeout 300 --timeout-method thread > $O/r04s_gpu_tests.log 2>&1 || { tail -60 $O/r04s_gpu_tests.log; exit 1; }
tail -3 $O/r04s_gpu_tests.log
