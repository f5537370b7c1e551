#!/bin/bash
# round 5, call x: register-tiled 8-stage strided pass (k_ntt_s8, the 2^21 LDE) -- LDE parity (2^21 natural and
# bit-reversed input), the 2^21-row-leaf compress node (GPU leaves vs oracle), LDE microbench vs the generic kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_prover.py "tests/test_compress_tree.py::test_gpu_mips_node_2e21_leaves" -m gpu > $O/r05x_tests.log 2>&1 || { tail -40 $O/r05x_tests.log; exit 1; }
tail -2 $O/r05x_tests.log
cat > /tmp/lde5.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 21, 67, 2)
print('generic8', os.environ.get('ZKM_NTT_GENERIC8', '0'), 'lde 2^21 x 67 %.3f ms' % d.bench_lde(1 << 21, 67, 10), flush=True)
PY
for i in 1 2 3; do
  for G in 0 1; do
    ZKM_NTT_GENERIC8=$G timeout -k 10 120 python3 /tmp/lde5.py >> $O/r05x_lde_ab.txt 2>&1 || { tail -20 $O/r05x_lde_ab.txt; exit 1; }
  done
done
cat $O/r05x_lde_ab.txt
