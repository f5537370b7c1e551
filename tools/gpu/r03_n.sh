#!/bin/bash
# round 3 (session 2): device tracegen GPU tests + tracegen bench; persistent prefetching strided NTT:
# parity with ZKM_NTT_PERSIST, then an A/B of the LDE stage
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_tracegen.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03n_tracegen.log 2>&1 || { tail -40 gpurun_out/r03n_tracegen.log; exit 1; }
tail -2 gpurun_out/r03n_tracegen.log
timeout -k 10 300 python3 -u bench.py --workload tracegen --steps 5 --warmup 1 > gpurun_out/r03n_tracegen_bench.json 2> gpurun_out/r03n_tracegen_bench.err || { tail -20 gpurun_out/r03n_tracegen_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03n_tracegen_bench.json'))
for k, v in d['chips'].items(): print(k, v['rows'], v['ms'], v['GBps'], v['frac_of_hbm_peak'])"
ZKM_NTT_PERSIST=2 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prover.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lde or ntt or 2e22" > gpurun_out/r03n_ntt_persist.log 2>&1 || { tail -40 gpurun_out/r03n_ntt_persist.log; exit 1; }
tail -2 gpurun_out/r03n_ntt_persist.log
for p in 0 1 2 0 1 2; do
  ZKM_NTT_PERSIST=$p timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-maxshape --no-pmc --steps 4 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stages_ms_per_shard']
print('persist $p: shard %.2f resident %.2f serial %.2f lde %.3f'%(d['ms_per_shard'], d['resident']['ms_per_shard'], d['serial_ms_per_shard'], s['lde']['ms_per_shard']))" | tee -a gpurun_out/r03n_ntt_ab.txt
done
