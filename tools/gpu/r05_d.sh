#!/bin/bash
# round 5, call d: the whole -m gpu suite after the node public-value semantics / shard PVs change (config
# parity first, incl. the 2^21-leaf node), then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=15 > $O/r05d_gpu_tests.log 2>&1 || { tail -60 $O/r05d_gpu_tests.log; exit 1; }
tail -3 $O/r05d_gpu_tests.log
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 2 > $O/r05d_bench.json 2> $O/r05d_bench.err || { tail -40 $O/r05d_bench.err; exit 1; }
tail -c 400 $O/r05d_bench.json
