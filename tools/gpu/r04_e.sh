#!/bin/bash
# round 4, call e: the Twirp Compress route end to end on the GPU, and an LDE column-batch sweep (does a
# batch whose work buffer fits the 256 MB Infinity Cache shorten the 2^22 LDE?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_service.py -m gpu > $O/r04e_service.log 2>&1 || { tail -30 $O/r04e_service.log; exit 1; }
tail -2 $O/r04e_service.log
cat > /tmp/ldecb.py <<PY
import os, sys; sys.path.insert(0, '$GRAFT_REPO_ROOT')
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 22, 67, 2)
print('cb', os.environ.get('ZKM_LDE_CB', 'default'), 'lde %.3f ms' % d.bench_lde(1 << 22, 67, 10), flush=True)
PY
for i in 1 2; do
  for cb in 1 2 4 8 16 32; do
    ZKM_LDE_CB=$cb timeout -k 10 120 python3 /tmp/ldecb.py >> $O/r04e_lde_cb.txt 2>&1 || { tail $O/r04e_lde_cb.txt; exit 1; }
  done
done
cat $O/r04e_lde_cb.txt
