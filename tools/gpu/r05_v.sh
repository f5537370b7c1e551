#!/bin/bash
# round 5, call v: strided plan A/B (ZKM_LDE_PLAN=1) over the smaller heights the recursion shards and short chips
# use (LDE microbench, blowup 2), alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
cat > /tmp/lde3.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
for logn, w in ((14, 128), (15, 128), (16, 128), (17, 128), (18, 128), (19, 67), (20, 67)):
    d.bench_lde(1 << logn, w, 2)
    print('plan', os.environ.get('ZKM_LDE_PLAN', '0'), 'lde 2^%d x %d %.4f ms' % (logn, w, d.bench_lde(1 << logn, w, 20)), flush=True)
PY
for i in 1 2; do
  for P in 0 1; do
    ZKM_LDE_PLAN=$P timeout -k 10 200 python3 /tmp/lde3.py >> $O/r05v_lde_ab.txt 2>&1 || { tail -20 $O/r05v_lde_ab.txt; exit 1; }
  done
done
sort -k5,5n -k2,2n $O/r05v_lde_ab.txt
