#!/bin/bash
# round 5, call j: openings with the prefetching dot-product kernel (k_open_dot_pf): proof bytes against the
# oracle, then the short fib line with ZKM_OPEN_PREFETCH=1 / 0 alternated (stage table: open_eval)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_prover.py -m gpu > $O/r05j_tests.log 2>&1 || { tail -30 $O/r05j_tests.log; exit 1; }
tail -3 $O/r05j_tests.log
for i in 1 2; do
  for pf in 1 0; do
    ZKM_OPEN_PREFETCH=$pf timeout -k 10 300 python3 bench.py --steps 4 --no-cpu-baseline --no-maxshape --no-compress --no-tendermint --no-sizes --no-pmc > $O/r05j_bench_$pf.json 2> $O/r05j_bench_$pf.err || { tail -20 $O/r05j_bench_$pf.err; exit 1; }
    python3 -c "
import json
d = json.loads(open('$O/r05j_bench_$pf.json').read().strip().splitlines()[-1])
st = d['stages_ms_per_shard']
print('prefetch $pf', 'open_eval', st['open_eval']['ms_per_shard'], 'fri_reduce', st['fri_reduce']['ms_per_shard'], 'open_total', st['open_total']['ms_per_shard'], 'resident', d['resident']['ms_per_shard'])
" | tee -a $O/r05j_ab.txt
  done
done
