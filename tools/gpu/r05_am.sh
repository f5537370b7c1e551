#!/bin/bash
# round 5, call am: t13 LDS addresses as base + constant stride (fused tile 121 -> 90 VGPRs, tile-major; 98 -> 66
# row-major) and the sequential-coset fused tile k_lde_fused13s (ZKM_T13_SEQ=1: 64 VGPRs, 34.8 KB LDS, four
# workgroups per CU instead of two) -- LDE parity with both, prover / blowup bytes, LDE microbench alternated,
# kernel traces of both
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_prover.py tests/test_blowup.py -m gpu > $O/r05am_tests.log 2>&1 || { tail -40 $O/r05am_tests.log; exit 1; }
echo "default: $(tail -1 $O/r05am_tests.log)"
ZKM_T13_SEQ=1 timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_prover.py -m gpu -k "lde or bytes_identical" > $O/r05am_tests_seq.log 2>&1 || { tail -40 $O/r05am_tests_seq.log; exit 1; }
echo "SEQ=1: $(tail -1 $O/r05am_tests_seq.log)"
cat > /tmp/ldeam.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
tag = 'seq' if os.environ.get('ZKM_T13_SEQ') == '1' else 'pair'
for logn, w in ((20, 67), (21, 67), (22, 64), (22, 67)):
    d.bench_lde(1 << logn, w, 2)
    print(tag, 'lde 2^%d x %d %.4f ms' % (logn, w, d.bench_lde(1 << logn, w, 20)), flush=True)
PY
for i in 1 2 3; do
  for S in 0 1; do
    ZKM_T13_SEQ=$S timeout -k 10 200 python3 /tmp/ldeam.py >> $O/r05am_lde_ab.txt 2>&1 || { tail -20 $O/r05am_lde_ab.txt; exit 1; }
  done
done
sort -k3,3 -k5,5 -k1,1 $O/r05am_lde_ab.txt
cd /tmp
for S in 0 1; do
  ZKM_T13_SEQ=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05am_prof$S -o kt -- python3 /tmp/ldeam.py > $O/r05am_prof$S.log 2>&1 || { tail -20 $O/r05am_prof$S.log; exit 1; }
  f=$(find $O/r05am_prof$S -name "*kernel_stats.csv" | head -1)
  cp $f $O/r05am_kernel_stats_seq$S.csv
  python3 - $O/r05am_kernel_stats_seq$S.csv $S <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'fused13' in r['Name'] or 's9b' in r['Name']:
        print('SEQ=%s %-50s calls %4s avg %9.0f ns' % (sys.argv[2], r['Name'].split('(')[0][11:], r['Calls'], float(r['AverageNs'])))
PY
done
