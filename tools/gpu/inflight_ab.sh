# headline in-flight count A/B (3 vs 4 vs 2), alternating runs
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/inf
cd $R
for i in 1 2; do
  for k in 3 4 2; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 1 --inflight $k --no-cpu-baseline --no-pmc > gpurun_out/inf/b_${k}_$i.json 2> gpurun_out/inf/b_${k}_$i.err || { tail -20 gpurun_out/inf/b_${k}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/inf/b_${k}_$i.json').read().strip().splitlines()[-1])
print('inflight=$k run=$i', 'value', d['value'], 'ms/shard', d['ms_per_shard'], 'resident', d['resident']['ms_per_shard'])"
  done
done
