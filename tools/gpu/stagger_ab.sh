# host-trace headline with / without staggered first copies (alternating runs)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/stag
cd $R
for i in 1 2 3; do
  for b in 0 1; do
    ZKM_NO_STAGGER=$((1-b)) timeout -k 10 300 python -u bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/stag/b_${b}_$i.json 2> gpurun_out/stag/b_${b}_$i.err || { tail -20 gpurun_out/stag/b_${b}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/stag/b_${b}_$i.json').read().strip().splitlines()[-1])
print('stagger=$b run=$i', 'value', d['value'], 'ms/shard', d['ms_per_shard'], 'resident', d['resident']['ms_per_shard'])"
  done
done
