#!/bin/bash
# round 3: GPU suite after the fused FRI transcript / fold+leaves and the faster 16-lane permutation;
# FRI timeline; LogUp look-ahead at 2 waves/SIMD; bench with the SQ pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h_tests.log 2>&1 || { tail -30 gpurun_out/r03h_tests.log; exit 1; }
tail -2 gpurun_out/r03h_tests.log
bash tools/gpu/fri_timeline.sh r03h || exit $?
cd "$GRAFT_REPO_ROOT"
for la in 40 56 48; do
  ZKM_JIT_LOOKAHEAD_P=$la timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-maxshape --no-pmc --steps 4 > gpurun_out/la.json 2> gpurun_out/la.err || { tail -5 gpurun_out/la.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/la.json')); s=d['stages_ms_per_shard']
print('look $la: shard %.2f serial %.2f fri_commit %.3f fri_reduce %.3f perm %.3f nodes %.3f'%(d['ms_per_shard'], d['serial_ms_per_shard'], s['fri_commit_phase']['ms_per_shard'], s['fri_reduce']['ms_per_shard'], s['perm_trace']['ms_per_shard'], s['merkle_nodes']['ms_per_shard']))" | tee -a gpurun_out/r03h_look.txt
done
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err
