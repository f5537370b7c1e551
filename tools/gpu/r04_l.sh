#!/bin/bash
# round 4, call l: the strided-tile access-pattern probe, tile-major LDE intermediates (parity + A/B), and
# whether a resident run earlier in the process slows the host-trace runs after it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 tools/probe/tile_probe > $O/r04l_tile_probe.txt 2>&1 || { cat $O/r04l_tile_probe.txt; exit 1; }
cat $O/r04l_tile_probe.txt
ZKM_LDE_TILED=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_blowup.py -m gpu -k "lde or blowup or commit" > $O/r04l_tiled_tests.log 2>&1 || { tail -30 $O/r04l_tiled_tests.log; exit 1; }
tail -2 $O/r04l_tiled_tests.log
cat > /tmp/ldeab.py <<PY
import os, sys; sys.path.insert(0, '$GRAFT_REPO_ROOT')
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 22, 67, 2)
print('tiled', os.environ.get('ZKM_LDE_TILED', '0'), 'lde %.3f ms' % d.bench_lde(1 << 22, 67, 10), flush=True)
PY
for i in 1 2 3; do
  for v in 0 1; do
    ZKM_LDE_TILED=$v timeout -k 10 120 python3 /tmp/ldeab.py >> $O/r04l_tiled_ab.txt 2>&1 || { tail $O/r04l_tiled_ab.txt; exit 1; }
  done
done
cat $O/r04l_tiled_ab.txt
for spec in "pipelined,pipelined 0 10 pipelined" "pipelined,pipelined 0 10 resident"; do
  echo "== $spec" >> $O/r04l_order.txt
  timeout -k 10 400 python3 -u tools/h2d_order.py $spec >> $O/r04l_order.txt 2>&1 || { tail -20 $O/r04l_order.txt; exit 1; }
done
echo "== DMA probe (copies as pipelined, proofs from the resident traces), warm-up resident" >> $O/r04l_order.txt
ZKM_BENCH_DMA_PROBE=1 timeout -k 10 400 python3 -u tools/h2d_order.py pipelined,pipelined 0 10 resident >> $O/r04l_order.txt 2>&1 || { tail -20 $O/r04l_order.txt; exit 1; }
grep -v amdgpu.ids $O/r04l_order.txt
