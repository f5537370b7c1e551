#!/bin/bash
# round 3 (session 2): LDE column batch at 2^22 (FibCpu headline): 16 vs 8 vs 4 vs 2 columns per batch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cb in 16 8 4 2 16 8 4 2; do
  export ZKM_LDE_CB=$cb
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-maxshape --no-pmc --steps 4 > gpurun_out/xb.json 2> gpurun_out/xb.err || { tail -5 gpurun_out/xb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/xb.json')); s=d['stages_ms_per_shard']
print('cb=$cb: shard %.2f resident %.2f serial %.2f lde %.3f'%(d['ms_per_shard'], d['resident']['ms_per_shard'], d['serial_ms_per_shard'], s['lde']['ms_per_shard']))" | tee -a gpurun_out/r03x_cb22_ab.txt
done
