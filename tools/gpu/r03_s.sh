#!/bin/bash
# round 3 (session 2): A/B of the extension-field product (8 vs 10 reductions): libzkm_hip_efnew.so vs the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in new old new old; do
  if [ $lib = new ]; then export ZKM_LIB=$GRAFT_REPO_ROOT/zkmips_amd/libzkm_hip_efnew.so; else unset ZKM_LIB; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-maxshape --no-pmc --steps 4 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stages_ms_per_shard']
print('ef $lib: shard %.2f resident %.2f serial %.2f perm %.3f quot %.3f fri_reduce %.3f open %.3f fri_commit %.3f'%(d['ms_per_shard'], d['resident']['ms_per_shard'], d['serial_ms_per_shard'], s['perm_trace']['ms_per_shard'], s['quotient']['ms_per_shard'], s['fri_reduce']['ms_per_shard'], s['open_eval']['ms_per_shard'], s['fri_commit_phase']['ms_per_shard']))" | tee -a gpurun_out/r03s_ef_ab.txt
done
export ZKM_LIB=$GRAFT_REPO_ROOT/zkmips_amd/libzkm_hip_efnew.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prover.py -m gpu -x -q --timeout 250 --timeout-method thread -k "2e22 or identical" > gpurun_out/r03s_parity.log 2>&1 || { tail -30 gpurun_out/r03s_parity.log; exit 1; }
tail -2 gpurun_out/r03s_parity.log
