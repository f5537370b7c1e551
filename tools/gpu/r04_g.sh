#!/bin/bash
# round 4, call g: native recursion runtime + compact compress witnesses (device event-row traces); GPU tests of
# the recursion / compress / service paths, node timing, then the default bench line (compress leg, host-trace
# copy waits)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_recursion.py tests/test_compress_tree.py tests/test_compress_verify.py tests/test_service.py -m gpu > $O/r04g_gpu_tests.log 2>&1 || { tail -30 $O/r04g_gpu_tests.log; exit 1; }
tail -2 $O/r04g_gpu_tests.log
timeout -k 10 300 python3 -u tools/compress_node_timing.py > $O/r04g_node_timing.txt 2>&1 || { tail -30 $O/r04g_node_timing.txt; exit 1; }
cat $O/r04g_node_timing.txt
timeout -k 10 900 python3 -u bench.py --steps 10 --warmup 2 > $O/r04g_bench.log 2>&1 || { tail -30 $O/r04g_bench.log; exit 1; }
tail -1 $O/r04g_bench.log | cut -c1-300
