#!/bin/bash
# round 5, call k: LDE microbench kernel breakdown, tile-major intermediates on / off (ZKM_LDE_TILED)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
cat > /tmp/lde1.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 22, 64, 2)
print('tiled', os.environ.get('ZKM_LDE_TILED', '1'), 'lde 2^22x64 %.3f ms' % d.bench_lde(1 << 22, 64, 10), flush=True)
PY
cd /tmp
for T in 1 0; do
  ZKM_LDE_TILED=$T timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05k_lde$T -o lde -- python3 /tmp/lde1.py > $O/r05k_lde$T.log 2>&1 || { tail -20 $O/r05k_lde$T.log; exit 1; }
  grep "lde 2" $O/r05k_lde$T.log
  find $O/r05k_lde$T -name "*kernel_stats.csv" -exec cp {} $O/r05k_lde${T}_stats.csv \;
  python3 - <<PY
import csv
for r in csv.DictReader(open("$O/r05k_lde${T}_stats.csv")):
    print("  ", r["Name"].split("(")[0][-40:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["MinNs"]) / 1e3, 1))
PY
done
