#!/bin/bash
# round 3 (session 2): adaptive LDE column batch (default) vs the fixed 16 -- parity, then compress A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_blowup.py tests/test_recursion.py tests/test_gpu_prover.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03v_parity.log 2>&1 || { tail -30 gpurun_out/r03v_parity.log; exit 1; }
tail -2 gpurun_out/r03v_parity.log
for cb in d 16 d 16 d 16; do
  if [ $cb = d ]; then unset ZKM_LDE_CB; else export ZKM_LDE_CB=$cb; fi
  timeout -k 10 300 python3 bench.py --workload compress --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cab.json 2> gpurun_out/cab.err || { tail -5 gpurun_out/cab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cab.json').read().strip().splitlines()[-1])
print('cb=$cb: proofs/s %.2f ms/proof %.3f serial %.3f'%(d['value'], d['ms_per_proof'], d['serial_ms_per_proof']))" | tee -a gpurun_out/r03v_cb_ab.txt
done
