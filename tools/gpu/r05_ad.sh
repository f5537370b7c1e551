#!/bin/bash
# round 5, call ad: LDE column batches small enough for the intermediates to stay in the 256 MiB Infinity Cache
# (ZKM_LDE_CB = 16 / 8 / 4 / 2 columns per batch), with the intermediate stores non-temporal (default library) or
# default-policy (libzkm_hip_ab.so, -DZKM_LDE_MID_AUX=0); LDE parity at CB=4 and CB=2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for CB in 4 2; do
  ZKM_LDE_CB=$CB timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "lde" > $O/r05ad_tests_cb$CB.log 2>&1 || { tail -40 $O/r05ad_tests_cb$CB.log; exit 1; }
  echo "CB=$CB: $(tail -1 $O/r05ad_tests_cb$CB.log)"
done
ZKM_LIB=$R/zkmips_amd/libzkm_hip_ab.so ZKM_LDE_CB=4 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "lde" > $O/r05ad_tests_ab.log 2>&1 || { tail -40 $O/r05ad_tests_ab.log; exit 1; }
echo "ab lib CB=4: $(tail -1 $O/r05ad_tests_ab.log)"
cat > /tmp/ldead.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
tag = ('midT' if 'ab' in os.environ.get('ZKM_LIB', '') else 'midNT') + ' cb' + os.environ.get('ZKM_LDE_CB', 'd')
for logn, w in ((22, 64), (22, 67), (21, 67)):
    d.bench_lde(1 << logn, w, 2)
    print(tag, 'lde 2^%d x %d %.4f ms' % (logn, w, d.bench_lde(1 << logn, w, 20)), flush=True)
PY
for i in 1 2; do
  for CB in 16 8 4 2; do
    ZKM_LDE_CB=$CB timeout -k 10 200 python3 /tmp/ldead.py >> $O/r05ad_lde_ab.txt 2>&1 || { tail -20 $O/r05ad_lde_ab.txt; exit 1; }
    ZKM_LIB=$R/zkmips_amd/libzkm_hip_ab.so ZKM_LDE_CB=$CB timeout -k 10 200 python3 /tmp/ldead.py >> $O/r05ad_lde_ab.txt 2>&1 || { tail -20 $O/r05ad_lde_ab.txt; exit 1; }
  done
done
sort -k4,4 -k6,6 -k1,2 $O/r05ad_lde_ab.txt
