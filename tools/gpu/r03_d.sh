#!/bin/bash
# round 3: compress tree over real leaves, the full-height SHA shard, the tendermint-shaped execution, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py --workload compress --leaf-log 14 --steps 1 --warmup 0 > gpurun_out/r03d_compress.json 2> gpurun_out/r03d_compress.err || exit $?
timeout -k 10 300 python3 -u -m pytest tests/test_syscall.py -k full_global_height -m gpu -v --timeout 290 --timeout-method thread > gpurun_out/r03d_sha_full.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py --workload tendermint --sigs 8 --tm-sha-blocks 64 --steps 1 --warmup 1 > gpurun_out/r03d_tendermint.json 2> gpurun_out/r03d_tendermint.err || exit $?
timeout -k 10 420 python3 bench.py > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err
