# k_compress_level look-ahead A/B (ZKM_CL_NODES=1: one node per thread, as before; 4: grid-stride with look-ahead)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cl
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_prover.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cl/tests.log 2>&1 || { tail -30 gpurun_out/cl/tests.log; exit 1; }
tail -1 gpurun_out/cl/tests.log
for i in 1 2; do
  for k in 1 4 8; do
    ZKM_CL_NODES=$k timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/cl/b_${k}_$i.json 2> gpurun_out/cl/b_${k}_$i.err || { tail -20 gpurun_out/cl/b_${k}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/cl/b_${k}_$i.json').read().strip().splitlines()[-1]); st=d['stages_ms_per_shard']
print('nodes=$k run=$i', 'merkle_nodes', st['merkle_nodes'], 'serial', d['serial_ms_per_shard'], 'resident', d['resident']['ms_per_shard'], 'value', d['value'])"
  done
done
