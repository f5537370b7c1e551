# LogUp JIT: waves-per-SIMD register cap x inversion group x lookahead: bash tools/gpu/perm_waves_sweep.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "0 10 48" "2 10 48" "2 5 48" "2 10 32" "2 5 24"; do
  set -- $cfg
  ZKM_JIT_PERM_WAVES=$1 ZKM_JIT_PERM_GROUP=$2 ZKM_JIT_LOOKAHEAD_P=$3 timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-maxshape --no-pmc --steps 4 > gpurun_out/pw.json 2> gpurun_out/pw.err || { tail -5 gpurun_out/pw.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/pw.json')); s=d['stages_ms_per_shard']
print('waves $1 group $2 look $3: shard %.2f serial %.2f perm %.3f'%(d['ms_per_shard'], d['serial_ms_per_shard'], s['perm_trace']['ms_per_shard']))" | tee -a gpurun_out/perm_waves_sweep.txt
done
