# LogUp JIT: batches per shared inversion x load lookahead (stage times from bench): bash tools/gpu/perm_group_sweep.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "10 48" "5 48" "5 24" "3 24" "2 16"; do
  set -- $cfg
  ZKM_JIT_PERM_GROUP=$1 ZKM_JIT_LOOKAHEAD_P=$2 timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-maxshape --steps 4 > gpurun_out/pg.json 2> gpurun_out/pg.err || { tail -5 gpurun_out/pg.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/pg.json')); s=d['stages_ms_per_shard']
print('group $1 look $2: step %.2f quot %.3f perm %.3f'%(d['ms_per_shard'], s['quotient']['ms_per_shard'], s['perm_trace']['ms_per_shard']))" | tee -a gpurun_out/perm_group_sweep.txt
done
