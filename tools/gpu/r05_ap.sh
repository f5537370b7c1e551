#!/bin/bash
# round 5, call ap: LDE column batch sweep on the final kernels (sequential-coset tile, default-policy intermediates):
# ZKM_LDE_CB = 4 / 8 / 16 / 32 at 2^20, 2^21, 2^22, alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
cat > /tmp/ldeap.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
tag = 'cb' + os.environ.get('ZKM_LDE_CB', 'default')
for logn, w in ((20, 67), (21, 67), (22, 67)):
    d.bench_lde(1 << logn, w, 2)
    print(tag, 'lde 2^%d x %d %.4f ms' % (logn, w, d.bench_lde(1 << logn, w, 20)), flush=True)
PY
for i in 1 2; do
  for CB in 4 8 16 32; do
    ZKM_LDE_CB=$CB timeout -k 10 200 python3 /tmp/ldeap.py >> $O/r05ap_lde_cb.txt 2>&1 || { tail -20 $O/r05ap_lde_cb.txt; exit 1; }
  done
  timeout -k 10 200 python3 /tmp/ldeap.py >> $O/r05ap_lde_cb.txt 2>&1 || { tail -20 $O/r05ap_lde_cb.txt; exit 1; }
done
sort -k3,3 -k5,5 -k1,1 $O/r05ap_lde_cb.txt
