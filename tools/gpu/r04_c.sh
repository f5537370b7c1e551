#!/bin/bash
# round 4, call c: two-column strided NTT tiles (k_ntt_s9c) parity + A/B against k_ntt_s9b, then the full
# default bench line (value = resident; sizes, maximal shape, compress and tendermint legs, CPU baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
ZKM_NTT_S9C=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_blowup.py -m gpu -k "lde or blowup or commit" > $O/r04c_s9c_tests.log 2>&1 || { tail -30 $O/r04c_s9c_tests.log; exit 1; }
tail -2 $O/r04c_s9c_tests.log
cat > /tmp/ldeab.py <<PY
import os, sys; sys.path.insert(0, '$GRAFT_REPO_ROOT')
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 22, 67, 2)
print(os.environ.get('ZKM_NTT_S9C', '0'), 'lde %.3f ms' % d.bench_lde(1 << 22, 67, 10), flush=True)
PY
for i in 1 2 3; do
  for v in 0 1; do
    ZKM_NTT_S9C=$v timeout -k 10 120 python3 /tmp/ldeab.py >> $O/r04c_lde_ab.txt 2>&1 || { tail $O/r04c_lde_ab.txt; exit 1; }
  done
done
cat $O/r04c_lde_ab.txt
timeout -k 10 900 python3 -u bench.py --steps 10 --warmup 2 > $O/r04c_bench.log 2>&1 || { tail -30 $O/r04c_bench.log; exit 1; }
tail -1 $O/r04c_bench.log | cut -c1-300
