#!/bin/bash
# round 5, call p: non-temporal stores in the strided NTT passes (libzkm_hip_ab.so, -DZKM_NTT_STORE_AUX=2) vs the
# default build: LDE microbench alternated, then the short fib line with each library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
R=$GRAFT_REPO_ROOT
cat > /tmp/lde1.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 22, 64, 2)
print(os.path.basename(os.environ.get('ZKM_LIB', 'default')), 'lde 2^22x64 %.3f ms' % d.bench_lde(1 << 22, 64, 10), flush=True)
PY
for i in 1 2 3; do
  timeout -k 10 120 python3 /tmp/lde1.py >> $O/r05p_lde_ab.txt 2>&1 || { tail -20 $O/r05p_lde_ab.txt; exit 1; }
  ZKM_LIB=$R/zkmips_amd/libzkm_hip_ab.so timeout -k 10 120 python3 /tmp/lde1.py >> $O/r05p_lde_ab.txt 2>&1 || { tail -20 $O/r05p_lde_ab.txt; exit 1; }
done
cat $O/r05p_lde_ab.txt
for L in "" "$R/zkmips_amd/libzkm_hip_ab.so" "" "$R/zkmips_amd/libzkm_hip_ab.so"; do
  ZKM_LIB=$L timeout -k 10 300 python3 bench.py --steps 4 --no-cpu-baseline --no-maxshape --no-compress --no-tendermint --no-sizes --no-pmc > $O/r05p_bench.json 2> $O/r05p_bench.err || { tail -20 $O/r05p_bench.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('$O/r05p_bench.json').read().strip().splitlines()[-1])
st = d['stages_ms_per_shard']
print('${L:+nt}', 'resident', d['resident']['ms_per_shard'], 'value', round(d['value']), {k: st[k]['ms_per_shard'] for k in ('lde', 'merkle_leaves', 'quotient')})
"
done
# the maximal shape's serial stage table (its own line)
timeout -k 10 600 python3 bench.py --workload maxshape --steps 3 --no-cpu-baseline --no-pmc > $O/r05p_maxshape.json 2> $O/r05p_maxshape.err || { tail -20 $O/r05p_maxshape.err; exit 1; }
python3 -c "
import json
d = json.loads(open('$O/r05p_maxshape.json').read().strip().splitlines()[-1])
st = d['stages_ms_per_shard']
print('maxshape', d['value'], d.get('ms_per_shard'), d.get('serial_ms_per_shard'), {k: v['ms_per_shard'] for k, v in st.items()})
"
