#!/bin/bash
# round 3: NTT parity after the XCD-aware strided remap, remap A/B, LogUp inversion-group sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_blowup.py -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1 || exit $?
for ab in remap noremap remap noremap; do
  if [ $ab = noremap ]; then export ZKM_NTT_NOREMAP=1; else unset ZKM_NTT_NOREMAP; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-maxshape --steps 4 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stages_ms_per_shard']; n=d['ntt']['hbm_measured']
print('$ab: shard %.2f serial %.2f lde %.3f ntt_bytes %.3e ratio %.2f'%(d['ms_per_shard'], d['serial_ms_per_shard'], s['lde']['ms_per_shard'], n['bytes_per_shard'], n['bytes_per_shard']/n['algorithmic_bytes_per_shard']))" | tee -a gpurun_out/r03e_remap_ab.txt
done
unset ZKM_NTT_NOREMAP
bash tools/gpu/perm_group_sweep.sh
