#!/bin/bash
# round 5, call y: register-tiled strided passes for 6..8 stages (k_ntt_sr) -- LDE parity (natural and bit-reversed
# input, 2^19 / 2^20 with the balanced plan / 2^21), blowup-4, prover bytes, the 2^21-leaf node; LDE microbench
# against the generic kernel (ZKM_NTT_GENERIC8=1) and, at 2^20, against the 9-stage-first plan
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_prover.py tests/test_blowup.py "tests/test_compress_tree.py::test_gpu_mips_node_2e21_leaves" -m gpu > $O/r05y_tests.log 2>&1 || { tail -40 $O/r05y_tests.log; exit 1; }
tail -1 $O/r05y_tests.log
ZKM_LDE_PLAN=0 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "lde" > $O/r05y_tests_plan0.log 2>&1 || { tail -40 $O/r05y_tests_plan0.log; exit 1; }
echo "plan 0: $(tail -1 $O/r05y_tests_plan0.log)"
cat > /tmp/lde6.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
tag = 'generic' if os.environ.get('ZKM_NTT_GENERIC8') == '1' else 'sr'
tag += ' plan' + os.environ.get('ZKM_LDE_PLAN', 'default')
for logn, w in ((17, 128), (18, 128), (19, 67), (20, 67), (21, 67)):
    d.bench_lde(1 << logn, w, 2)
    print(tag, 'lde 2^%d x %d %.4f ms' % (logn, w, d.bench_lde(1 << logn, w, 20)), flush=True)
PY
for i in 1 2; do
  for G in 0 1; do
    ZKM_NTT_GENERIC8=$G timeout -k 10 200 python3 /tmp/lde6.py >> $O/r05y_lde_ab.txt 2>&1 || { tail -20 $O/r05y_lde_ab.txt; exit 1; }
  done
  ZKM_LDE_PLAN=0 timeout -k 10 200 python3 /tmp/lde6.py >> $O/r05y_lde_ab.txt 2>&1 || { tail -20 $O/r05y_lde_ab.txt; exit 1; }
done
sort -k5,5 -k1,2 $O/r05y_lde_ab.txt
