#!/bin/bash
# round 3: GPU suite after in-kernel opening weights / FRI-reduce inverses / subtree Merkle levels /
# LogUp register cap; FRI timeline; subtree A/B; bench with the SQ pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g_tests.log 2>&1 || { tail -30 gpurun_out/r03g_tests.log; exit 1; }
tail -2 gpurun_out/r03g_tests.log
bash tools/gpu/fri_timeline.sh r03g || exit $?
cd "$GRAFT_REPO_ROOT"
for ab in sub nosub sub nosub; do
  if [ $ab = nosub ]; then export ZKM_NO_SUBTREE=1; else unset ZKM_NO_SUBTREE; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-maxshape --no-pmc --steps 4 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stages_ms_per_shard']
print('$ab: shard %.2f serial %.2f fri_commit %.3f nodes %.3f open %.3f fri_reduce %.3f perm %.3f'%(d['ms_per_shard'], d['serial_ms_per_shard'], s['fri_commit_phase']['ms_per_shard'], s['merkle_nodes']['ms_per_shard'], s['open_eval']['ms_per_shard'], s['fri_reduce']['ms_per_shard'], s['perm_trace']['ms_per_shard']))" | tee -a gpurun_out/r03g_subtree_ab.txt
done
unset ZKM_NO_SUBTREE
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/r03g_bench.json 2> gpurun_out/r03g_bench.err
