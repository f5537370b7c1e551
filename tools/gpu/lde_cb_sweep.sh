# LDE column-batch sweep (ZKM_LDE_CB): serial lde stage ms and resident ms/shard per setting
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cb
cd $R
for cb in 16 8 4 2; do
  ZKM_LDE_CB=$cb timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/cb/b_$cb.json 2> gpurun_out/cb/b_$cb.err || { tail -20 gpurun_out/cb/b_$cb.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/cb/b_$cb.json').read().strip().splitlines()[-1])
st=d['stages_ms_per_shard']; print('cb=$cb', 'lde', st.get('lde'), 'value', d['value'], 'resident', d['resident']['ms_per_shard'], 'serial', d['serial_ms_per_shard'])"
done
