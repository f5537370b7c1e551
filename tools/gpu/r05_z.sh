#!/bin/bash
# round 5, call z: wave-local L32 <-> L2 exchanges in the fused LDE tile (7 -> 2 workgroup barriers) -- LDE parity
# and prover bytes, then the LDE microbench against the barrier form (ZKM_T13_BARRIERS=1), alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_prover.py tests/test_blowup.py -m gpu > $O/r05z_tests.log 2>&1 || { tail -40 $O/r05z_tests.log; exit 1; }
tail -1 $O/r05z_tests.log
cat > /tmp/ldez.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
tag = 'barriers' if os.environ.get('ZKM_T13_BARRIERS') == '1' else 'wavelocal'
for logn, w in ((20, 67), (21, 67), (22, 64), (22, 67)):
    d.bench_lde(1 << logn, w, 2)
    print(tag, 'lde 2^%d x %d %.4f ms' % (logn, w, d.bench_lde(1 << logn, w, 20)), flush=True)
PY
for i in 1 2 3; do
  for B in 0 1; do
    ZKM_T13_BARRIERS=$B timeout -k 10 200 python3 /tmp/ldez.py >> $O/r05z_lde_ab.txt 2>&1 || { tail -20 $O/r05z_lde_ab.txt; exit 1; }
  done
done
sort -k3,3 -k1,1 $O/r05z_lde_ab.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05z_prof -o kt -- python3 /tmp/ldez.py > $O/r05z_prof.log 2>&1 || { tail -20 $O/r05z_prof.log; exit 1; }
find $O/r05z_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/r05z_kernel_stats.csv
python3 - <<PY
import csv
for r in csv.DictReader(open('$O/r05z_kernel_stats.csv')):
    if 'fused13' in r['Name'] or 'ntt_s' in r['Name']:
        print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
