#!/bin/bash
# round 5, call ao: the row-major -> column-major transpose of the uploaded traces with 128-row / 512-thread blocks
# (512-B column segments; ZKM_TW_ROWS=128) vs 64-row / 256-thread: prover parity with 128, kernel traces of a short
# headline run with each, alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
ZKM_TW_ROWS=128 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_prover.py tests/test_gpu_kernels.py -m gpu > $O/r05ao_tests.log 2>&1 || { tail -40 $O/r05ao_tests.log; exit 1; }
echo "TW_ROWS=128: $(tail -1 $O/r05ao_tests.log)"
cd /tmp
for i in 1 2; do
  for T in 64 128; do
    ZKM_TW_ROWS=$T timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05ao_prof$T-$i -o kt -- python3 $R/bench.py --steps 4 --warmup 1 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline > $O/r05ao_b$T-$i.json 2> $O/r05ao_b$T-$i.err || { tail -20 $O/r05ao_b$T-$i.err; exit 1; }
    f=$(find $O/r05ao_prof$T-$i -name "*kernel_stats.csv" | head -1)
    python3 - $f $T $i <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'to_col_major' in r['Name']:
        print('rows %s run %s %-45s calls %5s avg %9.1f us total %8.1f ms' % (sys.argv[2], sys.argv[3], r['Name'][:45], r['Calls'], float(r['AverageNs']) / 1e3, float(r['TotalDurationNs']) / 1e6))
PY
  done
done
