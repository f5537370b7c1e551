#!/bin/bash
# round 5, call c: strided LDE passes with register-generated twiddles -- parity, then LDE A/B against the
# loaded-twiddle form (ZKM_NTT_TWLOAD=1), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_blowup.py tests/test_gpu_prover.py -m gpu > $O/r05c_tests.log 2>&1 || { tail -30 $O/r05c_tests.log; exit 1; }
tail -1 $O/r05c_tests.log
cat > /tmp/ldeab.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 22, 67, 2)
print('twload', os.environ.get('ZKM_NTT_TWLOAD', '0'), 'lde %.3f ms' % d.bench_lde(1 << 22, 67, 10),
      '2^23x67 %.3f ms' % d.bench_lde(1 << 23, 67, 5), flush=True)
PY
: > $O/r05c_lde_ab.txt
for i in 1 2 3; do
  timeout -k 10 120 python3 /tmp/ldeab.py >> $O/r05c_lde_ab.txt 2>&1 || { tail $O/r05c_lde_ab.txt; exit 1; }
  ZKM_NTT_TWLOAD=1 timeout -k 10 120 python3 /tmp/ldeab.py >> $O/r05c_lde_ab.txt 2>&1 || { tail $O/r05c_lde_ab.txt; exit 1; }
done
grep lde $O/r05c_lde_ab.txt
