#!/bin/bash
# round 5, call o: quotient kernels with the factored point twiddle (JIT source change): the whole -m gpu suite
# (every machine's quotient through proof bytes), then the short fib line (stage table)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread > $O/r05o_gpu_tests.log 2>&1 || { tail -60 $O/r05o_gpu_tests.log; exit 1; }
tail -2 $O/r05o_gpu_tests.log
for i in 1 2; do
timeout -k 10 300 python3 bench.py --steps 4 --no-cpu-baseline --no-maxshape --no-compress --no-tendermint --no-sizes --no-pmc > $O/r05o_bench.json 2> $O/r05o_bench.err || { tail -20 $O/r05o_bench.err; exit 1; }
python3 -c "
import json
d = json.loads(open('$O/r05o_bench.json').read().strip().splitlines()[-1])
st = d['stages_ms_per_shard']
print('resident', d['resident']['ms_per_shard'], 'value', d['value'], {k: st[k]['ms_per_shard'] for k in ('quotient', 'lde', 'open_eval', 'fri_reduce', 'merkle_leaves')})
"
done
