#!/bin/bash
# round 5, call m: fused LDE tile with the twiddles loaded one phase ahead and LDS-only barriers: LDE parity
# (kernel tests + 2^22 proof bytes), LDE microbench kernel breakdown, short fib line (stage table)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_prover.py -m gpu > $O/r05m_tests.log 2>&1 || { tail -30 $O/r05m_tests.log; exit 1; }
tail -2 $O/r05m_tests.log
cat > /tmp/lde1.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 22, 64, 2)
print('lde 2^22x64 %.3f ms' % d.bench_lde(1 << 22, 64, 10), flush=True)
PY
for i in 1 2; do timeout -k 10 120 python3 /tmp/lde1.py; done
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05m_lde -o lde -- python3 /tmp/lde1.py > $O/r05m_lde.log 2>&1 || { tail -20 $O/r05m_lde.log; exit 1; }
find $O/r05m_lde -name "*kernel_stats.csv" -exec cp {} $O/r05m_lde_stats.csv \;
python3 - <<PY
import csv
for r in csv.DictReader(open("$O/r05m_lde_stats.csv")):
    print("  ", r["Name"].split("(")[0][-40:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["MinNs"]) / 1e3, 1))
PY
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --steps 4 --no-cpu-baseline --no-maxshape --no-compress --no-tendermint --no-sizes --no-pmc > $O/r05m_bench.json 2> $O/r05m_bench.err || { tail -20 $O/r05m_bench.err; exit 1; }
python3 -c "
import json
d = json.loads(open('$O/r05m_bench.json').read().strip().splitlines()[-1])
st = d['stages_ms_per_shard']
print('value', d['value'], 'resident', d['resident']['ms_per_shard'], 'lde', st['lde']['ms_per_shard'], 'open_eval', st['open_eval']['ms_per_shard'], 'serial', d['serial_ms_per_shard'])
"
