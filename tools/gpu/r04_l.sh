#!/bin/bash
# round 4, call l: (1) the strided-tile access-pattern probe; (2) tile-major LDE intermediates (parity + A/B);
# (3) the Montgomery multiply as plain C instead of inline asm (the compiler interleaves it: fewer s_nop
# hazard stalls; libzkm_hip_plain.so via ZKM_LIB) -- parity + LDE and resident A/B; (4) does a resident run
# earlier in the process slow the host-trace runs after it?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
PL=$GRAFT_REPO_ROOT/zkmips_amd/libzkm_hip_plain.so
timeout -k 10 120 tools/probe/tile_probe > $O/r04l_tile_probe.txt 2>&1 || { cat $O/r04l_tile_probe.txt; exit 1; }
cat $O/r04l_tile_probe.txt
ZKM_LDE_TILED=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_blowup.py -m gpu -k "lde or blowup or commit" > $O/r04l_tiled_tests.log 2>&1 || { tail -30 $O/r04l_tiled_tests.log; exit 1; }
tail -1 $O/r04l_tiled_tests.log
ZKM_LIB=$PL timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_blowup.py tests/test_gpu_prover.py -m gpu > $O/r04l_plain_tests.log 2>&1 || { tail -30 $O/r04l_plain_tests.log; exit 1; }
tail -1 $O/r04l_plain_tests.log
cat > /tmp/ldeab.py <<PY
import os, sys; sys.path.insert(0, '$GRAFT_REPO_ROOT')
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 22, 67, 2)
print('tiled', os.environ.get('ZKM_LDE_TILED', '0'), 'lib', os.path.basename(os.environ.get('ZKM_LIB', 'default')), 'lde %.3f ms' % d.bench_lde(1 << 22, 67, 10), flush=True)
PY
for i in 1 2 3; do
  ZKM_LDE_TILED=0 timeout -k 10 120 python3 /tmp/ldeab.py >> $O/r04l_lde_ab.txt 2>&1 || { tail $O/r04l_lde_ab.txt; exit 1; }
  ZKM_LDE_TILED=1 timeout -k 10 120 python3 /tmp/ldeab.py >> $O/r04l_lde_ab.txt 2>&1 || { tail $O/r04l_lde_ab.txt; exit 1; }
  ZKM_LIB=$PL ZKM_LDE_TILED=0 timeout -k 10 120 python3 /tmp/ldeab.py >> $O/r04l_lde_ab.txt 2>&1 || { tail $O/r04l_lde_ab.txt; exit 1; }
  ZKM_LIB=$PL ZKM_LDE_TILED=1 timeout -k 10 120 python3 /tmp/ldeab.py >> $O/r04l_lde_ab.txt 2>&1 || { tail $O/r04l_lde_ab.txt; exit 1; }
done
cat $O/r04l_lde_ab.txt
for i in 1 2; do
  echo "default" >> $O/r04l_shard_ab.txt
  timeout -k 10 300 python3 -u tools/h2d_attrib.py resident 8 >> $O/r04l_shard_ab.txt 2>&1 || { tail -20 $O/r04l_shard_ab.txt; exit 1; }
  echo "plain mad" >> $O/r04l_shard_ab.txt
  ZKM_LIB=$PL timeout -k 10 300 python3 -u tools/h2d_attrib.py resident 8 >> $O/r04l_shard_ab.txt 2>&1 || { tail -20 $O/r04l_shard_ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/r04l_shard_ab.txt
for spec in "pipelined,pipelined 0 10 pipelined" "pipelined,pipelined 0 10 resident"; do
  echo "== $spec" >> $O/r04l_order.txt
  timeout -k 10 400 python3 -u tools/h2d_order.py $spec >> $O/r04l_order.txt 2>&1 || { tail -20 $O/r04l_order.txt; exit 1; }
done
grep -v amdgpu.ids $O/r04l_order.txt
