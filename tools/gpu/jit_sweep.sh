# quotient/perm JIT load-lookahead sweep (stage times from bench): bash tools/gpu/jit_sweep.sh
set -e
mkdir -p gpurun_out
for q in 4 8 12 16; do
  ZKM_JIT_LOOKAHEAD_Q=$q ZKM_JIT_LOOKAHEAD_P=$((q*6)) timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/js.json 2> gpurun_out/js.err || { tail -5 gpurun_out/js.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/js.json')); s=d['stages_ms_per_step']
print('q $q p $((q*6)): step %.2f quot %.3f perm %.3f'%(d['ms_per_step'], s['quotient']['ms_per_step'], s['perm_trace']['ms_per_step']))"
done
