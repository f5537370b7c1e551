#!/bin/bash
# round 3 (session 2): blowup-4 LDE with one shared inverse transform -- parity, then compress A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_blowup.py tests/test_recursion.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03t_parity.log 2>&1 || { tail -30 gpurun_out/r03t_parity.log; exit 1; }
tail -2 gpurun_out/r03t_parity.log
for sh in 1 0 1 0; do
  export ZKM_LDE4_SHARED=$sh
  timeout -k 10 300 python3 bench.py --workload compress --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cab.json 2> gpurun_out/cab.err || { tail -5 gpurun_out/cab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cab.json').read().strip().splitlines()[-1])
print('shared=$sh: proofs/s %.2f ms/proof %.3f serial %.3f'%(d['value'], d['ms_per_proof'], d['serial_ms_per_proof']))" | tee -a gpurun_out/r03t_lde4_ab.txt
done
