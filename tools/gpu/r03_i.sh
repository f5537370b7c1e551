#!/bin/bash
# round 3: EC precompiles + Ed25519 (refactored gadgets) GPU parity; subtree threshold sweep;
# compress tree over real leaves; full-height SHA shard; tendermint execution
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_ec_precompiles.py tests/test_edwards.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/r03i_tests.log 2>&1 || { tail -30 gpurun_out/r03i_tests.log; exit 1; }
tail -3 gpurun_out/r03i_tests.log
for sub in 8192 16384 65536 32768; do
  ZKM_SUB16=$sub timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-maxshape --no-pmc --steps 4 > gpurun_out/sb.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb.json')); s=d['stages_ms_per_shard']
print('sub16 $sub: shard %.2f serial %.2f fri_commit %.3f nodes %.3f'%(d['ms_per_shard'], d['serial_ms_per_shard'], s['fri_commit_phase']['ms_per_shard'], s['merkle_nodes']['ms_per_shard']))" | tee -a gpurun_out/r03i_sub16.txt
done
timeout -k 10 500 python3 -u bench.py --workload compress --leaf-log 14 --steps 1 --warmup 0 > gpurun_out/r03i_compress.json 2> gpurun_out/r03i_compress.err || { tail -5 gpurun_out/r03i_compress.err; exit 1; }
timeout -k 10 300 python3 -u -m pytest tests/test_syscall.py -k full_global_height -m gpu -v --timeout 290 --timeout-method thread > gpurun_out/r03i_sha_full.log 2>&1 || { tail -20 gpurun_out/r03i_sha_full.log; exit 1; }
timeout -k 10 400 python3 bench.py --workload tendermint --sigs 8 --tm-sha-blocks 64 --steps 1 --warmup 1 > gpurun_out/r03i_tendermint.json 2> gpurun_out/r03i_tendermint.err
