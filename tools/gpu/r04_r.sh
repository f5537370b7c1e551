#!/bin/bash
# round 4, call r: compress witnesses through /dev/shm, warmed witness workers: the compress / service GPU
# tests, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_compress_tree.py tests/test_service.py tests/test_compress_verify.py -m gpu -v --timeout 300 --timeout-method thread > $O/r04r_gpu_tests.log 2>&1 || { tail -40 $O/r04r_gpu_tests.log; exit 1; }
tail -2 $O/r04r_gpu_tests.log
timeout -k 10 1000 python3 -u bench.py > $O/r04r_bench.log 2>&1 || { tail -30 $O/r04r_bench.log; exit 1; }
tail -1 $O/r04r_bench.log | cut -c1-300
ls /dev/shm | grep -c zkm_ || true
