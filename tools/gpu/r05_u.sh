#!/bin/bash
# round 5, call u: strided plan A/B (ZKM_LDE_PLAN=1: one 9-stage buffer-addressed pass, the fused tile taking the
# rest) -- LDE parity under both plans at 2^10..2^23, LDE microbench per size alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
for P in 0 1; do
  ZKM_LDE_PLAN=$P timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "lde" > $O/r05u_tests_$P.log 2>&1 || { tail -30 $O/r05u_tests_$P.log; exit 1; }
  echo "plan $P: $(tail -1 $O/r05u_tests_$P.log)"
done
cat > /tmp/lde2.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
for logn, w in ((20, 67), (21, 67), (23, 32)):
    d.bench_lde(1 << logn, w, 2)
    print('plan', os.environ.get('ZKM_LDE_PLAN', '0'), 'lde 2^%d x %d %.3f ms' % (logn, w, d.bench_lde(1 << logn, w, 10)), flush=True)
PY
for i in 1 2; do
  for P in 0 1; do
    ZKM_LDE_PLAN=$P timeout -k 10 200 python3 /tmp/lde2.py >> $O/r05u_lde_ab.txt 2>&1 || { tail -20 $O/r05u_lde_ab.txt; exit 1; }
  done
done
cat $O/r05u_lde_ab.txt
