#!/bin/bash
# round 5, call ac: k_ntt_sr for 5-stage strided passes (the 2^18 LDE's pass and both of the 2^23 LDE's) -- LDE
# parity (2^18 / 2^23 natural, 2^18 bit-reversed input) and prover bytes, then the LDE microbench against the
# LDS-staged generic kernel (ZKM_NTT_GENERIC8=1), alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_prover.py tests/test_blowup.py -m gpu > $O/r05ac_tests.log 2>&1 || { tail -40 $O/r05ac_tests.log; exit 1; }
tail -1 $O/r05ac_tests.log
cat > /tmp/ldeac.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
tag = 'generic' if os.environ.get('ZKM_NTT_GENERIC8') == '1' else 'sr'
for logn, w in ((18, 128), (23, 16), (23, 64)):
    d.bench_lde(1 << logn, w, 2)
    print(tag, 'lde 2^%d x %d %.4f ms' % (logn, w, d.bench_lde(1 << logn, w, 20)), flush=True)
PY
for i in 1 2 3; do
  for G in 0 1; do
    ZKM_NTT_GENERIC8=$G timeout -k 10 200 python3 /tmp/ldeac.py >> $O/r05ac_lde_ab.txt 2>&1 || { tail -20 $O/r05ac_lde_ab.txt; exit 1; }
  done
done
sort -k3,3 -k5,5 -k1,1 $O/r05ac_lde_ab.txt
