#!/bin/bash
# round 3: compress tree over real leaves (nodes verify their children), the node GPU test, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_compress_verify.py -m gpu -v --timeout 280 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1 || exit $?
timeout -k 10 500 python3 -u bench.py --workload compress --leaf-log 14 --steps 1 --warmup 0 > gpurun_out/r03c_compress.json 2> gpurun_out/r03c_compress.err || exit $?
timeout -k 10 420 python3 bench.py > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err
