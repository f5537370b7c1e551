#!/bin/bash
# round 5, call g: NTT built with the plain-C Montgomery product (the compiler schedules it; the asm form costs
# ~700 s_nop hazards in k_lde_fused13) vs the default build: LDE microbench alternated, its kernel breakdown
# with the plain build, and the short fib bench line with each library
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
d.bench_lde(1 << 22, 67, 2)
print(os.environ.get('ZKM_LIB', 'default'), 'lde 2^22x67 %.3f ms' % d.bench_lde(1 << 22, 67, 10), flush=True)
PY
for i in 1 2; do
  timeout -k 10 120 python3 /tmp/lde1.py >> $O/r05g_lde_ab.txt 2>&1 || { tail -20 $O/r05g_lde_ab.txt; exit 1; }
  ZKM_LIB=$R/zkmips_amd/libzkm_hip_ab.so timeout -k 10 120 python3 /tmp/lde1.py >> $O/r05g_lde_ab.txt 2>&1 || { tail -20 $O/r05g_lde_ab.txt; exit 1; }
done
cat $O/r05g_lde_ab.txt
cd /tmp
ZKM_LIB=$R/zkmips_amd/libzkm_hip_ab.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05g_lde -o lde -- python3 /tmp/lde1.py > $O/r05g_lde.log 2>&1 || { tail -20 $O/r05g_lde.log; exit 1; }
find $O/r05g_lde -name "*kernel_stats.csv" -exec cp {} $O/r05g_lde_kernel_stats.csv \;
cd $R
for L in "" "$R/zkmips_amd/libzkm_hip_ab.so"; do
  ZKM_LIB=$L timeout -k 10 400 python3 bench.py --steps 8 --no-cpu-baseline --no-maxshape --no-compress --no-tendermint --no-sizes --no-pmc > $O/r05g_bench_${L:+ab}.json 2> $O/r05g_bench_${L:+ab}.err || { tail -20 $O/r05g_bench_${L:+ab}.err; exit 1; }
  tail -c 600 $O/r05g_bench_${L:+ab}.json
done
