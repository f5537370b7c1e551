# host-trace headline with / without binding the host threads to the GPU's NUMA node (alternating runs)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/numa
cd $R
for i in 1 2; do
  for b in 0 1; do
    ZKM_NO_NUMA_BIND=$((1-b)) timeout -k 10 300 python -u bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/numa/b_${b}_$i.json 2> gpurun_out/numa/b_${b}_$i.err || { tail -20 gpurun_out/numa/b_${b}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/numa/b_${b}_$i.json').read().strip().splitlines()[-1])
print('bind=$b run=$i', 'value', d['value'], 'ms/shard', d['ms_per_shard'], 'resident', d['resident']['ms_per_shard'], d.get('host_threads_bound_to'))"
  done
done
