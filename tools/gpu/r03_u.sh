#!/bin/bash
# round 3 (session 2): compress-shape A/B of the LDE column batch (default 16 vs 64 vs all columns)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cb in 16 0 64 16 0 64; do
  export ZKM_LDE_CB=$cb
  timeout -k 10 300 python3 bench.py --workload compress --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cab.json 2> gpurun_out/cab.err || { tail -5 gpurun_out/cab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cab.json').read().strip().splitlines()[-1])
print('cb=$cb: proofs/s %.2f ms/proof %.3f serial %.3f'%(d['value'], d['ms_per_proof'], d['serial_ms_per_proof']))" | tee -a gpurun_out/r03u_cb_ab.txt
done
