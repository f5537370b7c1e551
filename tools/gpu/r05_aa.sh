#!/bin/bash
# round 5, call aa: persistent prefetching strided pass k_ntt_s9q (ZKM_NTT_PF = workgroups per CU) -- LDE parity with
# PF=2 and PF=1, then the LDE microbench PF 0 / 1 / 2 alternated, and a kernel trace of each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
for PF in 2 1; do
  ZKM_NTT_PF=$PF timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "lde" > $O/r05aa_tests_pf$PF.log 2>&1 || { tail -40 $O/r05aa_tests_pf$PF.log; exit 1; }
  echo "PF=$PF: $(tail -1 $O/r05aa_tests_pf$PF.log)"
done
ZKM_NTT_PF=2 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_prover.py -m gpu -k "bytes_identical" > $O/r05aa_prover_pf2.log 2>&1 || { tail -40 $O/r05aa_prover_pf2.log; exit 1; }
echo "prover PF=2: $(tail -1 $O/r05aa_prover_pf2.log)"
cat > /tmp/ldeaa.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
tag = 'pf' + os.environ.get('ZKM_NTT_PF', '0')
for logn, w in ((20, 67), (21, 67), (22, 64), (22, 67), (23, 16)):
    d.bench_lde(1 << logn, w, 2)
    print(tag, 'lde 2^%d x %d %.4f ms' % (logn, w, d.bench_lde(1 << logn, w, 20)), flush=True)
PY
for i in 1 2 3; do
  for PF in 0 1 2; do
    ZKM_NTT_PF=$PF timeout -k 10 200 python3 /tmp/ldeaa.py >> $O/r05aa_lde_ab.txt 2>&1 || { tail -20 $O/r05aa_lde_ab.txt; exit 1; }
  done
done
sort -k3,3 -k5,5 -k1,1 $O/r05aa_lde_ab.txt
cd /tmp
for PF in 0 2; do
  ZKM_NTT_PF=$PF timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05aa_prof$PF -o kt -- python3 /tmp/ldeaa.py > $O/r05aa_prof$PF.log 2>&1 || { tail -20 $O/r05aa_prof$PF.log; exit 1; }
done
for PF in 0 2; do
  f=$(find $O/r05aa_prof$PF -name "*kernel_stats.csv" | head -1)
  cp $f $O/r05aa_kernel_stats_pf$PF.csv
  python3 - $O/r05aa_kernel_stats_pf$PF.csv <<PY
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'ntt' in r['Name'] or 'fused' in r['Name']:
        print('$PF', r['Name'][:70], r['Calls'], r['AverageNs'], r['TotalDurationNs'])
PY
done
