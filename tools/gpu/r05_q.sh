#!/bin/bash
# round 5, call q: the fused LDE tile's stores non-temporal too (libzkm_hip_ab.so, -DZKM_FUSED13_NT_STORE) vs
# the default: LDE microbench alternated; then the LDE kernel tests with the default build (nt strided stores)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
R=$GRAFT_REPO_ROOT
cat > /tmp/lde1.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 22, 64, 2)
print(os.path.basename(os.environ.get('ZKM_LIB', 'default')), 'lde 2^22x64 %.3f ms' % d.bench_lde(1 << 22, 64, 10), flush=True)
PY
for i in 1 2 3; do
  timeout -k 10 120 python3 /tmp/lde1.py >> $O/r05q_lde_ab.txt 2>&1 || { tail -20 $O/r05q_lde_ab.txt; exit 1; }
  ZKM_LIB=$R/zkmips_amd/libzkm_hip_ab.so timeout -k 10 120 python3 /tmp/lde1.py >> $O/r05q_lde_ab.txt 2>&1 || { tail -20 $O/r05q_lde_ab.txt; exit 1; }
done
cat $O/r05q_lde_ab.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_prover.py tests/test_blowup.py -m gpu > $O/r05q_tests.log 2>&1 || { tail -30 $O/r05q_tests.log; exit 1; }
tail -2 $O/r05q_tests.log
