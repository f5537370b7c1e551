#!/bin/bash
# round 5, call w: LDE kernel breakdown at 2^21 x 67 (the reference's default shard height) and 2^23 x 32
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
for cfg in "21 67" "23 32"; do
set -- $cfg
cat > /tmp/lde4.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << $1, $2, 2)
print('lde 2^$1 x $2 %.3f ms' % d.bench_lde(1 << $1, $2, 10), flush=True)
PY
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05w_lde$1 -o lde -- python3 /tmp/lde4.py > $O/r05w_lde$1.log 2>&1 || { tail -20 $O/r05w_lde$1.log; exit 1; }
grep "lde 2" $O/r05w_lde$1.log
find $O/r05w_lde$1 -name "*kernel_stats.csv" -exec cp {} $O/r05w_lde$1_stats.csv \;
python3 - <<PY
import csv
for r in csv.DictReader(open("$O/r05w_lde$1_stats.csv")):
    print("  ", r["Name"].split("(")[0][-44:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["TotalDurationNs"]) / 1e6 / 12, 3), "ms/LDE")
PY
cd $GRAFT_REPO_ROOT
done
